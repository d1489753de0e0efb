"""Fused one-pass statistics (ops.moments): host path, Chan combination, and (GPU) the HIP kernel."""
import math

import pytest
import torch

from cuda_mpi_reductions_amd.ops import combine_moments, fill_, moments, synthetic


def ref(x):
    xd = x.double()
    return xd.mean().item(), xd.var(unbiased=False).item(), xd.min().item(), xd.max().item()


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("n", [1, 2, 7, 1000, 100_003])
def test_host_moments(dt, n):
    x = synthetic(n, dt, seed=n) * 5 - 2
    m = moments(x)
    mean, var, mn, mx = ref(x)
    assert m["count"] == n and m["min"] == mn and m["max"] == mx
    assert abs(m["mean"] - mean) <= 1e-12 * max(1, abs(mean))
    assert abs(m["var"] - var) <= 1e-9 * max(1e-12, var) + 1e-15


def test_shifted_variance_is_stable():
    # |mean| >> std: the naive Σx²/n - mean² loses every digit, the shifted form does not.
    x = synthetic(100_000, torch.float64) * 1e-3 + 1e9
    m = moments(x)
    assert abs(m["var"] - ref(x)[1]) <= 1e-6 * ref(x)[1]


def test_chan_combination_matches_whole():
    x = synthetic(10_000, torch.float64, seed=3)
    from cuda_mpi_reductions_amd.ops.moments import _raw
    a, b = _raw(x[:3333]), _raw(x[3333:])
    n, mean, m2, mn, mx = combine_moments(a, b)
    wm, wv, wmn, wmx = ref(x)
    assert n == 10_000 and abs(mean - wm) < 1e-12 and abs(m2 / n - wv) < 1e-12 and mn == wmn and mx == wmx


def test_rejects_ints():
    with pytest.raises(TypeError):
        moments(torch.arange(10))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.float64, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n", [1, 3, 63, 65, 4097, 1_000_003, (1 << 24) + 5])
def test_device_moments(dt, n):
    x = torch.empty(n, dtype=dt, device="cuda")
    fill_(x, "uniform", seed=n)
    x.mul_(7).sub_(3)
    m = moments(x)
    mean, var, mn, mx = ref(x)
    assert m["count"] == n and m["min"] == mn and m["max"] == mx
    assert abs(m["mean"] - mean) <= 1e-9 * max(1.0, abs(mean))
    assert abs(m["var"] - var) <= 1e-9 * max(1e-9, var)


@pytest.mark.gpu
def test_device_moments_misaligned_view():
    base = torch.empty(100_001, dtype=torch.float32, device="cuda")
    fill_(base, "uniform", seed=1)
    x = base[1:]
    m = moments(x)
    assert m["min"] == x.min().item() and abs(m["mean"] - x.double().mean().item()) < 1e-9
