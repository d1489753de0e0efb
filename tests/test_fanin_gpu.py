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


def _identity(dt, op):
    if op == "sum":
        return 0
    info = torch.iinfo(dt)
    return info.max if op == "min" else info.min


@pytest.mark.parametrize("dt,op", [(torch.float64, "sum"), (torch.int64, "sum"), (torch.int64, "min"),
                                   (torch.int64, "max"), (torch.int32, "max")])
def test_fanin_bound_reports_error_poisons_and_recovers(dt, op):
    from cuda_mpi_reductions_amd._native import native
    from cuda_mpi_reductions_amd.ops import Reducer, default_acc_dtype
    C = native()
    dev = torch.device("cuda", 0)
    n = 1 << 24
    x = torch.ones(n, dtype=dt, device=dev)
    x[n // 3] = 5 if op == "max" else -5  # the extreme sits in some workgroup's slice
    exp = {"sum": x.sum().item(), "min": -5, "max": 5}[op]
    red = Reducer(dev)
    out = torch.zeros(1, dtype=default_acc_dtype(dt, op), device=dev)
    plan = _launch(C, red, x, out, op)
    torch.cuda.synchronize()
    assert plan["single_pass"] and plan["grid"] > 1, plan
    assert out.item() == exp and red.check() is None and red.ws.error() == 0
    # workgroup 0 publishes 50 ms late against a 1 ms bound: reported, result poisoned — NaN for
    # floats, the operator's identity for integers (neutral in a cross-rank fold; ADVICE r3: not 0,
    # which wins a MIN over positive values) — and the error word is the signal
    out.fill_(7)
    _launch(C, red, x, out, op, fanin_bound_ticks=1 * TICKS_PER_MS, debug_delay_wg=0,
            debug_delay_ticks=50 * TICKS_PER_MS)
    torch.cuda.synchronize()
    got = out.item()
    assert red.ws.error() != 0

    def poisoned(v):
        return math.isnan(v) if dt.is_floating_point else v == _identity(out.dtype, op)
    assert poisoned(got), got
    # sticky: the next (good) launch is flagged too — its slots may hold the late store
    _launch(C, red, x, out, op)
    torch.cuda.synchronize()
    assert red.ws.error() != 0 and poisoned(out.item())
    msg = red.check()  # reports and resets
    assert msg is not None and "wait bound" in msg and red.ws.error() == 0
    # after the reset: exact again, many launches back to back (epochs advance, nothing cleared)
    for _ in range(50):
        _launch(C, red, x, out, op)
    torch.cuda.synchronize()
    assert out.item() == exp and red.check() is None


@pytest.mark.parametrize("dt,op", [(torch.float64, "sum"), (torch.int64, "min")])
def test_reduce_check_raises_on_fanin_error(dt, op):
    # a library caller asking for check=True gets an exception, not a silent
    # identity / NaN — through Reducer.__call__ and through ops.reduce (the default reducer)
    from cuda_mpi_reductions_amd._native import native
    from cuda_mpi_reductions_amd.ops import FaninError, Reducer, default_acc_dtype, reduce
    from cuda_mpi_reductions_amd.ops.reduce import _default_reducer
    C = native()
    dev = torch.device("cuda", 0)
    x = torch.ones(1 << 24, dtype=dt, device=dev)
    out = torch.zeros(1, dtype=default_acc_dtype(dt, op), device=dev)
    for red in (Reducer(dev), None):
        target = red if red is not None else (reduce(x, op), _default_reducer(dev))[1]
        _launch(C, target, x, out, op, fanin_bound_ticks=1 * TICKS_PER_MS, debug_delay_wg=0,
                debug_delay_ticks=50 * TICKS_PER_MS)
        with pytest.raises(FaninError, match="wait bound"):
            (red(x, op, check=True) if red is not None else reduce(x, op, check=True))
        # the check reset the workspace: the next checked call is exact
        got = red(x, op, check=True) if red is not None else reduce(x, op, check=True)
        assert got.item() == (x.sum().item() if op == "sum" else 1)


def _set_epoch(C, red, value):
    """Write the workspace's fan-in epoch counter (test hook via its device address)."""
    import numpy as np
    src = torch.from_numpy(np.array([value], dtype=np.uint32).view(np.int32)).to("cuda")
    C.memcpy_d2d(red.ws.fan_ptr, src.data_ptr(), 4, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()


def test_fanin_epoch_wrap_invalidates_old_slots():
    # the 32-bit epoch wraps; a slot last written a whole cycle earlier (beyond the grid
    # of every launch since) must not match the new cycle's tag. Slots beyond the small grid are
    # tagged with epoch 3 from array A; the counter is moved to just before the wrap, small launches
    # cross it, and a big launch of array B runs with epoch 3 again while the workgroup of one of
    # those slots publishes 20 ms late: it must be waited for, not replaced by A's stale partial.
    from cuda_mpi_reductions_amd._native import native
    from cuda_mpi_reductions_amd.ops import Reducer
    C = native()
    dev = torch.device("cuda", 0)
    a = torch.ones(1 << 26, dtype=torch.float64, device=dev)
    b = torch.full((1 << 26,), 2.0, dtype=torch.float64, device=dev)
    small = torch.ones(3_000_001, dtype=torch.float64, device=dev)
    red = Reducer(dev)
    outs = torch.zeros(8, dtype=torch.float64, device=dev)
    _set_epoch(C, red, 2)
    big_grid = _launch(C, red, a, outs[0:1])["grid"]  # epoch 3: every slot < big_grid tagged 3
    assert big_grid > 64
    _set_epoch(C, red, 0xFFFFFFFD)
    for i in range(1, 5):  # epochs 0xfffffffe, 0xffffffff (wrap: slots zeroed), 1, 2
        _launch(C, red, small, outs[i:i + 1], max_blocks=37)
    late = big_grid - 2  # beyond the small grid, not the finisher
    _launch(C, red, b, outs[5:6], debug_delay_wg=late, debug_delay_ticks=20 * TICKS_PER_MS)  # epoch 3
    torch.cuda.synchronize()
    exp = [float(a.numel())] + [float(small.numel())] * 4 + [2.0 * b.numel(), 0.0, 0.0]
    assert outs.tolist() == exp and red.check() is None


def test_xcd_anchor_across_the_epoch_wrap_single_and_two_pass(monkeypatch):
    # The XCD-weighted split's anchor (XcdAnchor) is tagged with the launch's fan-in epoch, which
    # the polled finisher or — two-pass — the finalize launch ends. Skewed launches of both kinds,
    # interleaved on one workspace and across the epoch's wrap (both ends zero the slots and the
    # anchor there): every result exact, no anchor wait ever timing out (error bit 2).
    from cuda_mpi_reductions_amd._native import native
    from cuda_mpi_reductions_amd.ops import Reducer
    monkeypatch.setenv("MIREDUCE_XCD_SKEW", "100")
    C = native()
    dev = torch.device("cuda", 0)
    n = 26_000_003
    g = torch.Generator(device="cpu").manual_seed(17)
    x = torch.randint(-(1 << 40), 1 << 40, (n,), generator=g, dtype=torch.int64).to(dev)
    exp = x.sum().item()
    red = Reducer(dev)
    outs = torch.zeros(8, dtype=torch.int64, device=dev)
    _set_epoch(C, red, 0xFFFFFFFB)
    for i in range(8):  # epochs 0xfffffffc .. 0xffffffff (wrap), 1, 2, 3, 4
        plan = _launch(C, red, x, outs[i:i + 1], single_pass=(i % 2 == 0))
        assert plan["xskew"] > 0 and plan["single_pass"] == (i % 2 == 0), plan
    torch.cuda.synchronize()
    assert outs.tolist() == [exp] * 8 and red.check() is None


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


@pytest.mark.parametrize("single_pass", [True, False], ids=["polled", "two_pass"])
@pytest.mark.parametrize("dt", [torch.float64, torch.int64])
def test_late_xcd_anchor_poisons_and_reports(dt, single_pass):
    # a workgroup that gives up waiting for the XCD anchor streams the parity-0
    # tail, which need not match its peers' — the split is no longer a bijection. The launch must
    # then be poisoned (NaN / the identity) and flagged (error bit 2, its own message), in both the
    # polled single-pass path and the two-pass path, and the launch after the reset is exact again.
    from cuda_mpi_reductions_amd._native import native
    from cuda_mpi_reductions_amd.ops import Reducer, default_acc_dtype
    C = native()
    dev = torch.device("cuda", 0)
    n = 26_000_003  # 208 MB of 8-byte elements: the window-4 plan with the anchored XCD skew
    g = torch.Generator(device="cpu").manual_seed(23)
    if dt.is_floating_point:
        x = torch.rand(n, generator=g, dtype=dt).to(dev)
    else:
        x = torch.randint(1, 1 << 30, (n,), generator=g, dtype=dt).to(dev)
    exp = x.sum().item()
    red = Reducer(dev)
    out = torch.zeros(1, dtype=default_acc_dtype(dt, "sum"), device=dev)
    # (208 MB is only ~25 rounds per workgroup: the default 20 permille rounds to no skew, so ask for 100)
    plan = _launch(C, red, x, out, single_pass=single_pass, fanin_bound_ticks=1 * TICKS_PER_MS,
                   debug_delay_anchor_ticks=20 * TICKS_PER_MS, xcd_skew=100)
    assert plan["xskew"] != 0 and plan["window"] == 4, plan
    torch.cuda.synchronize()
    word = red.ws.error()
    assert word & 2, word
    got = out.item()
    assert (math.isnan(got) if dt.is_floating_point else got == 0), got  # never a plausible wrong sum
    msg = red.check()
    assert msg is not None and "XCD anchor" in msg, msg
    _launch(C, red, x, out, single_pass=single_pass, xcd_skew=100)
    torch.cuda.synchronize()
    assert red.check() is None
    got = out.item()
    assert (abs(got - exp) <= 1e-9 * abs(exp) if dt.is_floating_point else got == exp), (got, exp)
