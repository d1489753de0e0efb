"""bfloat16 / float16 inputs (csrc/include/mireduce/half.hpp): an MI355X addition to the reference's
int/float/double (cuda/C/src/reduction/reduction_kernel.cu:527-564). The streaming kernel reads 8
elements per 16-byte load and accumulates in fp32; references are plain PyTorch fp64 reductions of
the same tensors.

CPU tests: conversions against torch for every 16-bit pattern, RNE rounding of the fill, host
reducer, the app's CLI rejections. GPU tests: every op x size x misalignment, device fill ==
host fill, NaN/inf semantics, every kernel variant, and the reduction app end to end.
"""
import math
import os

import pytest
import torch

from cuda_mpi_reductions_amd.ops import (KernelConfig, Reducer, cpu_reduce, default_acc_dtype, fill_, reduce,
                                         sum_tolerance, synthetic)
from helpers import BIN, ensure_built, run

HALVES = [torch.bfloat16, torch.float16]
IDS = ["bf16", "f16"]


@pytest.mark.parametrize("dt", HALVES, ids=IDS)
def test_default_accumulator_is_fp32(dt):
    for op in ("sum", "min", "max"):
        assert default_acc_dtype(dt, op) == torch.float32


@pytest.mark.parametrize("dt", HALVES, ids=IDS)
def test_every_bit_pattern_converts_like_torch(dt):
    x = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(dt)
    f = x.float()
    finite = torch.isfinite(f)
    # MIN / MAX of each single value returns it exactly (host conversion == torch's)
    vals = x[finite][::97]
    for v, ref in zip(vals, f[finite][::97]):
        got = cpu_reduce(v.reshape(1), "max")
        assert got == ref.item() or (got == 0.0 and ref.item() == 0.0), (v, got, ref)
    assert cpu_reduce(x[finite], "max") == f[finite].max().item()
    assert cpu_reduce(x[finite], "min") == f[finite].min().item()
    # NaN patterns are ignored by MIN/MAX (IEEE minNum/maxNum), like the other float types
    nan = x[torch.isnan(f)][:5]
    assert cpu_reduce(torch.cat([nan, torch.tensor([2.0], dtype=dt)]), "max") == 2.0


@pytest.mark.parametrize("dt", HALVES, ids=IDS)
def test_constant_fill_rounds_to_nearest_even(dt):
    g = torch.Generator().manual_seed(5)
    vals = torch.cat([
        torch.randn(300, generator=g) * 10.0 ** torch.randint(-9, 6, (300,), generator=g),
        torch.tensor([1.0 + 2.0 ** -8, 1.0 + 3 * 2.0 ** -8, 1.0 + 2.0 ** -11, 1.0 + 3 * 2.0 ** -11,
                      65504.0, 65519.0, 65520.0, 1e6, 2.0 ** -24, 2.0 ** -25, 3 * 2.0 ** -26, 6e-8, 1e-40, 0.0, -0.0]),
    ])
    for v in vals.tolist():
        x = torch.empty(3, dtype=dt)
        fill_(x, "constant", value=v)
        ref = torch.tensor([v], dtype=torch.float32).to(dt)
        assert x[0].view(torch.int16).item() == ref.view(torch.int16).item(), (v, x[0].item(), ref.item())


@pytest.mark.parametrize("dt", HALVES, ids=IDS)
@pytest.mark.parametrize("pattern", ["uniform", "smallint", "iotamod"])
def test_host_reducer(dt, pattern):
    x = synthetic(200_003, dt, pattern=pattern, seed=11)
    if pattern == "uniform":
        assert 0.0 <= x.float().min().item() and x.float().max().item() < 1.0  # never rounds up to 1
    exp = x.double().sum().item()
    got = cpu_reduce(x, "sum")
    assert abs(got - exp) <= 1e-6 * max(1.0, abs(exp))
    assert cpu_reduce(x, "min") == x.float().min().item()
    assert cpu_reduce(x, "max") == x.float().max().item()


def test_half_plan_uses_tuned_point():
    from cuda_mpi_reductions_amd._native import native
    C = native()
    for code in (4, 5):  # bf16, f16 at 8 GB and 1 GB (profiles/r3_types/)
        for n in (4_000_000_000, 500_000_000):
            p = C.plan(0, n, code)  # SUM: 256 x 8, 1 WG/CU, window 4
            assert (p["block"], p["unroll"], p["grid"], p["nontemporal"], p["window"]) == (256, 8, 256, True, 4), \
                (code, n, p)
            p = C.plan(0, n, code, op=2)  # MAX: 256 x 8, 2 WG/CU, window 2
            assert (p["block"], p["unroll"], p["grid"], p["nontemporal"], p["window"]) == (256, 8, 512, True, 2), \
                (code, n, p)


def test_reduction_app_rejects_ladder_for_half():
    ensure_built()
    r = run([os.path.join(BIN, "reduction"), "--method=SUM", "--type=bf16", "--kernel=6", "--n=1000"])
    assert r.returncode != 0 and "bf16/half use kernels 7/8" in (r.stdout + r.stderr)


def test_cross_rank_apps_reject_half():
    ensure_built()
    r = run([os.path.join(BIN, "reduce_mpi"), "--dtypes=bf16"])
    assert r.returncode != 0 and "16-bit" in (r.stdout + r.stderr)


# ------------------------------------------------------------------------------------------ GPU

DEV = "cuda:0"
SIZES = [1, 7, 8, 9, 63, 64, 65, 511, 512, 513, 4097, 65537, 1_000_003, (1 << 22) + 5]


def _check(got, x, op):
    xd = x.double()
    if op == "sum":
        exp = xd.sum().item()
        tol = sum_tolerance(x.dtype, torch.float32, x.numel(), xd.abs().sum().item())
        assert abs(got - exp) <= tol, (got, exp, tol)
    elif op == "min":
        assert got == xd.min().item()
    else:
        assert got == xd.max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("dt", HALVES, ids=IDS)
@pytest.mark.parametrize("op", ["sum", "min", "max"])
@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("misalign", [0, 1, 3])
def test_gpu_half_sizes(dt, op, n, misalign):
    base = torch.empty(n + misalign, dtype=dt, device=DEV)
    fill_(base, "uniform", seed=n + 31 * misalign)
    x = base[misalign:]
    if op != "sum":  # plant the extreme somewhere that is not the first tile
        x[(n * 5) // 7] = -3.5 if op == "min" else 7.25
    out = reduce(x, op)
    assert out.dtype == torch.float32
    _check(out.item(), x, op)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", HALVES, ids=IDS)
def test_gpu_half_device_fill_matches_host(dt):
    for pattern in ("uniform", "smallint", "iotamod"):
        d = synthetic(1_000_001, dt, device=DEV, pattern=pattern, seed=9, offset=12345)
        h = synthetic(1_000_001, dt, pattern=pattern, seed=9, offset=12345)
        assert torch.equal(d.cpu().view(torch.int16), h.view(torch.int16)), pattern


@pytest.mark.gpu
@pytest.mark.parametrize("dt", HALVES, ids=IDS)
def test_gpu_half_nan_inf(dt):
    x = torch.zeros(100_000, dtype=dt, device=DEV)
    x[777] = float("nan")
    x[50_000] = 4.0
    assert reduce(x, "max").item() == 4.0  # NaN ignored by maxNum
    assert math.isnan(reduce(x, "sum").item())
    x[777] = float("inf")
    assert reduce(x, "max").item() == math.inf
    assert reduce(x, "sum").item() == math.inf
    x[778] = float("-inf")
    assert reduce(x, "min").item() == -math.inf


@pytest.mark.gpu
@pytest.mark.parametrize("dt", HALVES, ids=IDS)
def test_gpu_half_every_variant(dt):
    x = synthetic(3_000_017, dt, device=DEV, seed=4)
    r = Reducer(DEV)
    for block in (256, 512, 1024):
        for unroll in (2, 4, 8, 16):
            for nt in (False, True):
                cfg = KernelConfig(block=block, unroll=unroll, nontemporal=nt)
                _check(r(x, "sum", config=cfg).item(), x, "sum")
                _check(r(x, "max", config=cfg).item(), x, "max")
    _check(r(x, "sum", config=KernelConfig(single_pass=False)).item(), x, "sum")


@pytest.mark.gpu
@pytest.mark.parametrize("ty", ["bf16", "half"])
def test_gpu_reduction_app_half(ty):
    ensure_built()
    for method in ("SUM", "MIN", "MAX"):
        r = run([os.path.join(BIN, "reduction"), f"--method={method}", f"--type={ty}", "--n=33554437",
                 "--iterations=5", "--qatest"])
        assert r.returncode == 0, r.stdout + r.stderr
        assert "&&&& PASSED" in r.stdout + r.stderr
        assert "GPU result" in r.stdout


def test_host_reducer_does_not_saturate():
    """fp32-accumulated host sums are compensated in fp64: a float-typed Neumaier sum of 40M ones
    saturates (sum and compensation both stall at 2^24) — the bug that made a 4e9-element bf16 check
    report 64.0 for a true 237.5."""
    x = torch.ones(40_000_000, dtype=torch.bfloat16)
    assert cpu_reduce(x, "sum", threads=1) == 40_000_000.0
    y = torch.full((40_000_000,), 1.0, dtype=torch.float32)
    assert cpu_reduce(y, "sum", torch.float32, threads=1) == 40_000_000.0
