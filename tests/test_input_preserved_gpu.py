"""In-place safety of every reduction path ("run an in-place-safety test for any
multi-pass path"). The reference's multi-pass loop reduces its partials in place in d_odata
(reduction.cpp:344-357) — harmless there because the input lives in d_idata, but a multi-pass or
scratch-reusing path that wrote into its input, or a tail/head lane that stored past a view's end,
would corrupt user data silently. Each case reduces a misaligned view inside a guarded buffer and
then checks, bit for bit, that the view AND the guard elements on both sides are unchanged."""
import pytest
import torch

from cuda_mpi_reductions_amd.ops import (KernelConfig, Reducer, arg_reduce, fill_, ladder_reduce, moments, norm,
                                         reduce, reduce_dim, reduce_many, reduce_partials)

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
GUARD = 4099  # elements on each side of the view (odd: the view starts misaligned)


def _guarded(n: int, dt: torch.dtype, seed: int):
    base = torch.empty(n + 2 * GUARD, dtype=dt, device=DEV)
    fill_(base, "uniform" if dt.is_floating_point else "fullrange", seed=seed)
    return base, base[GUARD:GUARD + n]


def _bits(t: torch.Tensor) -> torch.Tensor:
    return t.view({1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[t.element_size()]).clone()


def _assert_preserved(base: torch.Tensor, snap: torch.Tensor):
    torch.cuda.synchronize()
    now = _bits(base)
    bad = (now != snap).nonzero()
    assert bad.numel() == 0, f"{bad.numel()} elements changed, first at {bad[0].item() - GUARD} relative to the view"


DTYPES = [torch.float64, torch.float32, torch.int32, torch.int64, torch.bfloat16]


@pytest.mark.parametrize("dt", DTYPES, ids=str)
@pytest.mark.parametrize("n", [1, 1000, 1_000_003, 40_000_003])  # the last: > 192 MB plans (window) for 8 bytes
def test_streaming_reduce_single_and_two_pass(dt, n):
    base, x = _guarded(n, dt, seed=n)
    snap = _bits(base)
    for op in ("sum", "min", "max"):
        reduce(x, op)
        reduce(x, op, config=KernelConfig(single_pass=False))
        reduce_partials(x, op)
    r = Reducer(DEV)
    bound = r.bind(x, "sum")
    bound.launch(torch.cuda.current_stream(DEV).cuda_stream)
    _assert_preserved(base, snap)


@pytest.mark.parametrize("kernel", range(7))
def test_ladder_multi_pass(kernel):
    # the ladder relaunches on its own partials until one value is left (ping-pong scratch)
    base, x = _guarded(3_333_331, torch.float64, seed=kernel)
    snap = _bits(base)
    for op in ("sum", "min", "max"):
        for threads in (64, 256):
            ladder_reduce(x, op, kernel=kernel, threads=threads)
    _assert_preserved(base, snap)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.int64], ids=str)
def test_axis_list_arg_and_moment_paths(dt):
    rows, cols = 1537, 2049
    base, flat = _guarded(rows * cols, dt, seed=7)
    x = flat.view(rows, cols)
    snap = _bits(base)
    for op in ("sum", "min", "max"):
        reduce_dim(x, op, dim=1)
        reduce_dim(x, op, dim=0)
    reduce_many([x[:100], x[100:900], x[900:]], "sum")
    for op in ("max", "min"):
        arg_reduce(x, op)
        arg_reduce(x, op, dim=1)
    if dt.is_floating_point:
        norm(flat)
        norm(flat, float("inf"))
        moments(flat)
    _assert_preserved(base, snap)
