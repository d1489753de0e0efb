"""Polled fan-in of the single-pass kernel (csrc/kernels/reduce_kernels.hpp): epoch-tagged slots and
the sticky error word. A workgroup delayed past the finisher's wait bound (test
hook ReduceConfig::debug_delay_wg / debug_delay_ticks, bound fanin_bound_ticks) must yield a reported
error and a poisoned result — never a plausible-looking fold of unpublished slots — the error must stay
sticky until the host reset, and the launch after the reset must be exact again. Reference pattern:
threadFenceReduction_kernel.cu:137-167 (the retirement counter is reset, so no stale state leaks
into the next launch)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

TICKS_PER_MS = 100_000  # gfx950 wall clock: 100 MHz


def _launch(C, red, x, out, op="sum", **kw):
    from cuda_mpi_reductions_amd.ops import default_acc_dtype, dtype_code, op_code
    acc = default_acc_dtype(x.dtype, op)
    return C.reduce(red.ws, x.data_ptr(), x.numel(), dtype_code(x.dtype), op_code(op), dtype_code(acc),
                    out.data_ptr(), torch.cuda.current_stream().cuda_stream, **kw)


@pytest.mark.parametrize("dt", [torch.float64, torch.int64])
def test_fanin_bound_reports_error_poisons_and_recovers(dt):
    from cuda_mpi_reductions_amd._native import native
    from cuda_mpi_reductions_amd.ops import Reducer
    C = native()
    dev = torch.device("cuda", 0)
    n = 1 << 24
    x = torch.ones(n, dtype=dt, device=dev)
    red = Reducer(dev)
    out = torch.zeros(1, dtype=dt, device=dev)
    plan = _launch(C, red, x, out)
    torch.cuda.synchronize()
    assert plan["poll"] and plan["grid"] > 1, plan
    assert out.item() == n and red.check() is None and red.ws.error() == 0
    # workgroup 0 publishes 50 ms late against a 1 ms bound: reported, result poisoned
    out.fill_(7)
    _launch(C, red, x, out, fanin_bound_ticks=1 * TICKS_PER_MS, debug_delay_wg=0,
            debug_delay_ticks=50 * TICKS_PER_MS)
    torch.cuda.synchronize()
    got = out.item()
    assert red.ws.error() != 0
    assert (math.isnan(got) if dt.is_floating_point else got == 0), got  # NaN / the SUM identity
    # sticky: the next (good) launch is flagged too — its slots may hold the late store
    _launch(C, red, x, out)
    torch.cuda.synchronize()
    assert red.ws.error() != 0 and (math.isnan(out.item()) if dt.is_floating_point else out.item() == 0)
    msg = red.check()  # reports and resets
    assert msg is not None and "wait bound" in msg and red.ws.error() == 0
    # after the reset: exact again, many launches back to back (epochs advance, nothing cleared)
    for _ in range(50):
        _launch(C, red, x, out)
    torch.cuda.synchronize()
    assert out.item() == n and red.check() is None


def test_fanin_slow_workgroup_within_bound_is_exact():
    # a straggler that publishes before the bound is simply waited for
    from cuda_mpi_reductions_amd._native import native
    from cuda_mpi_reductions_amd.ops import Reducer
    C = native()
    dev = torch.device("cuda", 0)
    x = torch.arange(1 << 22, dtype=torch.float64, device=dev)
    red = Reducer(dev)
    out = torch.zeros(1, dtype=torch.float64, device=dev)
    _launch(C, red, x, out, debug_delay_wg=3, debug_delay_ticks=5 * TICKS_PER_MS)
    torch.cuda.synchronize()
    assert out.item() == x.sum().item() and red.check() is None


def test_fanin_epochs_do_not_leak_between_grids():
    # alternate launches of different grids on one workspace: a slot left by the larger grid carries
    # an old epoch and must never be folded into the smaller grid's result
    from cuda_mpi_reductions_amd._native import native
    from cuda_mpi_reductions_amd.ops import Reducer
    C = native()
    dev = torch.device("cuda", 0)
    big = torch.ones(1 << 26, dtype=torch.float64, device=dev)
    small = torch.ones(3_000_001, dtype=torch.float64, device=dev)
    red = Reducer(dev)
    outs = torch.zeros(40, dtype=torch.float64, device=dev)
    grids = set()
    for i in range(40):
        x = big if i % 2 == 0 else small
        grids.add(_launch(C, red, x, outs[i:i + 1], max_blocks=0 if i % 2 == 0 else 37)["grid"])
    torch.cuda.synchronize()
    assert len(grids) == 2, grids
    exp = torch.tensor([float(big.numel()) if i % 2 == 0 else float(small.numel()) for i in range(40)],
                       dtype=torch.float64, device=dev)
    assert torch.equal(outs, exp) and red.check() is None
