"""Numerics of the native HIP reduction kernels vs plain PyTorch fp64/int64 references.

Closes the reference's test gaps: every (op x dtype x accumulator), sizes
around wavefront/tile/grid boundaries, misaligned base pointers (the min/max OOB bug B1/B2 of
reduction_kernel.cu:140,157), >2^31 elements (bug B4), every compiled kernel variant, the
two-kernel path as an oracle for the single-pass path, and back-to-back launches (fan-in epochs).
"""
import math

import pytest
import torch

from cuda_mpi_reductions_amd._native import native
from cuda_mpi_reductions_amd.ops import KernelConfig, Reducer, fill_, reduce, reduce_partials, sum_tolerance

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
COMBOS = [
    (torch.int32, "sum", torch.int64),
    (torch.int32, "sum", torch.int32),
    (torch.int32, "min", torch.int32),
    (torch.int32, "max", torch.int32),
    (torch.int64, "sum", torch.int64),
    (torch.int64, "min", torch.int64),
    (torch.int64, "max", torch.int64),
    (torch.float32, "sum", torch.float64),
    (torch.float32, "sum", torch.float32),
    (torch.float32, "min", torch.float32),
    (torch.float32, "max", torch.float32),
    (torch.float64, "sum", torch.float64),
    (torch.float64, "min", torch.float64),
    (torch.float64, "max", torch.float64),
]
SIZES = [1, 2, 3, 63, 64, 65, 255, 256, 257, 1023, 1024, 1025, 4097, 65537, 1_000_003, (1 << 22) + 7]


def expected(x: torch.Tensor, op: str, acc: torch.dtype):
    if op == "sum":
        if acc.is_floating_point:
            return x.double().sum().item(), x.double().abs().sum().item()
        if acc == torch.int32:  # wraps modulo 2^32
            s = x.long().sum().item() & 0xFFFFFFFF
            return (s - (1 << 32) if s >= (1 << 31) else s), 0.0
        return x.long().sum().item(), 0.0
    if op == "min":
        return x.min().item(), 0.0
    return x.max().item(), 0.0


def check(got, x, op, acc, n):
    exp, abs_sum = expected(x, op, acc)
    if op == "sum" and acc.is_floating_point:
        tol = sum_tolerance(x.dtype, acc, n, abs_sum)
        assert abs(got - exp) <= tol, (got, exp, tol)
    else:
        assert got == exp, (got, exp)


@pytest.mark.parametrize("dt,op,acc", COMBOS, ids=lambda v: str(v).replace("torch.", ""))
@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("misalign", [0, 1])
def test_all_combos_sizes(dt, op, acc, n, misalign):
    base = torch.empty(n + misalign, dtype=dt, device=DEV)
    fill_(base, "fullrange" if not dt.is_floating_point else "uniform", seed=n * 7 + misalign)
    x = base[misalign:]
    got = reduce(x, op, acc).item()
    check(got, x, op, acc, n)


def test_empty_gives_identity():
    for dt, op, acc in COMBOS:
        x = torch.empty(0, dtype=dt, device=DEV)
        got = reduce(x, op, acc).item()
        if op == "sum":
            assert got == 0
        elif op == "min":
            assert got == (math.inf if acc.is_floating_point else torch.iinfo(acc).max)
        else:
            assert got == (-math.inf if acc.is_floating_point else torch.iinfo(acc).min)


@pytest.mark.parametrize("block", [256, 512])
@pytest.mark.parametrize("unroll", [2, 4, 8])
@pytest.mark.parametrize("nt", [True, False])
@pytest.mark.parametrize("single_pass", [True, False])
def test_every_variant(block, unroll, nt, single_pass):
    n = 3_000_017
    x = torch.empty(n, dtype=torch.float64, device=DEV)
    fill_(x, "uniform", seed=11)
    r = Reducer(DEV, config=KernelConfig(block=block, unroll=unroll, nontemporal=nt, single_pass=single_pass))
    for op in ("sum", "min", "max"):
        check(r(x, op).item(), x, op, torch.float64, n)
    xi = torch.empty(n, dtype=torch.int64, device=DEV)
    fill_(xi, "fullrange", seed=12)
    for op in ("min", "max"):
        check(r(xi, op).item(), xi, op, torch.int64, n)


@pytest.mark.parametrize("max_blocks", [1, 2, 3, 7, 64, 0])
def test_grid_caps(max_blocks):
    # the polled fan-in over any grid: one workgroup (no fan-in), odd grids, the planner's own
    n = 5_000_011
    x = torch.empty(n, dtype=torch.int32, device=DEV)
    fill_(x, "fullrange", seed=3)
    r = Reducer(DEV, config=KernelConfig(max_blocks=max_blocks))
    check(r(x, "sum").item(), x, "sum", torch.int64, n)
    check(r(x, "max").item(), x, "max", torch.int32, n)


def test_back_to_back_launches_epochs():
    # 300 launches queued without host sync, each on different data: a stale slot (an earlier
    # launch's epoch) or a missing epoch advance would make some launch finalise early/never.
    n = 2_000_003
    r = Reducer(DEV)
    xs = [torch.empty(n, dtype=torch.int64, device=DEV) for _ in range(3)]
    for i, x in enumerate(xs):
        fill_(x, "fullrange", seed=100 + i)
    outs = torch.empty(300, dtype=torch.int64, device=DEV)
    for i in range(300):
        r(xs[i % 3], "sum", out=outs[i:i + 1])
    torch.cuda.synchronize()
    exp = [x.sum().item() for x in xs]
    got = outs.tolist()
    assert all(got[i] == exp[i % 3] for i in range(300))


def test_single_vs_two_pass_int_bitwise():
    n = 7_000_001
    x = torch.empty(n, dtype=torch.int64, device=DEV)
    fill_(x, "fullrange", seed=5)
    a = Reducer(DEV, config=KernelConfig(single_pass=True))(x, "sum").item()
    b = Reducer(DEV, config=KernelConfig(single_pass=False))(x, "sum").item()
    assert a == b == x.sum().item()


def test_partials_and_host_fold():
    C = native()
    n = 4_000_037
    x = torch.empty(n, dtype=torch.float64, device=DEV)
    fill_(x, "uniform", seed=9)
    for op in ("sum", "min", "max"):
        parts, plan = reduce_partials(x, op)
        host = parts.cpu()
        folded = C.cpu_reduce(host.data_ptr(), host.numel(), 3, {"sum": 0, "min": 1, "max": 2}[op], 3, 1)
        check(folded, x, op, torch.float64, n)


@pytest.mark.parametrize("dt", [torch.int32, torch.int64, torch.float32, torch.float64])
@pytest.mark.parametrize("pattern", ["uniform", "smallint", "fullrange", "iotamod", "constant"])
def test_device_fill_matches_host_fill(dt, pattern):
    n = 100_003
    d = torch.empty(n, dtype=dt, device=DEV)
    h = torch.empty(n, dtype=dt)
    fill_(d, pattern, seed=42, offset=12345, value=3.0)
    fill_(h, pattern, seed=42, offset=12345, value=3.0)
    assert torch.equal(d.cpu(), h)


@pytest.mark.parametrize("op", ["sum", "min", "max"])
def test_combine_elementwise(op):
    C = native()
    n = 1_000_005
    a = torch.empty(n, dtype=torch.float64, device=DEV)
    b = torch.empty(n, dtype=torch.float64, device=DEV)
    fill_(a, "uniform", seed=1)
    fill_(b, "uniform", seed=2)
    ref = {"sum": a + b, "min": torch.minimum(a, b), "max": torch.maximum(a, b)}[op]
    C.combine_elementwise(a.data_ptr(), b.data_ptr(), n, 3, {"sum": 0, "min": 1, "max": 2}[op],
                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(a, ref)


def test_more_than_2_pow_31_elements():
    # 2^31 + 17 int32 (8 GiB): 64-bit indexing end to end (reference: int size / unsigned bytes).
    n = (1 << 31) + 17
    x = torch.empty(n, dtype=torch.int32, device=DEV)
    fill_(x, "iotamod")
    got = reduce(x, "sum").item()
    full, rem = divmod(n, 1024)
    exp = full * (1023 * 1024 // 2) + rem * (rem - 1) // 2
    assert got == exp
    assert reduce(x, "max").item() == 1023
    assert reduce(x, "min").item() == 0
    del x
    torch.cuda.empty_cache()


def test_nan_and_inf_semantics():
    x = torch.tensor([1.0, float("nan"), -3.0, 2.0], dtype=torch.float64, device=DEV)
    # MIN/MAX ignore NaN (IEEE minNum/maxNum, same as std::fmin on the host); SUM propagates it.
    assert reduce(x, "min").item() == -3.0
    assert reduce(x, "max").item() == 2.0
    assert math.isnan(reduce(x, "sum").item())
    y = torch.tensor([1.0, float("inf"), -2.0], dtype=torch.float32, device=DEV)
    assert reduce(y, "max").item() == math.inf


# ---------------------------------------------------------------------------------------------
# Harris ladder kernels 0..6 (csrc/kernels/ladder.hip) — the reference's --kernel values.
from cuda_mpi_reductions_amd.ops import ladder_reduce  # noqa: E402

LADDER_COMBOS = [c for c in COMBOS if c[0] in (torch.int32, torch.float64, torch.int64)]


@pytest.mark.parametrize("kernel", range(7))
@pytest.mark.parametrize("dt,op,acc", LADDER_COMBOS, ids=lambda v: str(v).replace("torch.", ""))
@pytest.mark.parametrize("n", [1, 63, 65, 1000, 65537, 1_000_003])
def test_ladder_kernels(kernel, dt, op, acc, n):
    x = torch.empty(n, dtype=dt, device=DEV)
    fill_(x, "uniform" if dt.is_floating_point else "fullrange", seed=kernel * 31 + n)
    got = ladder_reduce(x, op, kernel=kernel, acc_dtype=acc).item()
    check(got, x, op, acc, n)


@pytest.mark.parametrize("threads", [64, 128, 256, 512, 1024])
@pytest.mark.parametrize("kernel", [0, 3, 4, 5, 6])
def test_ladder_block_sizes(threads, kernel):
    n = 3_333_331
    x = torch.empty(n, dtype=torch.float64, device=DEV)
    fill_(x, "uniform", seed=threads)
    for op in ("sum", "min", "max"):
        check(ladder_reduce(x, op, kernel=kernel, threads=threads).item(), x, op, torch.float64, n)


def test_ladder_kernel6_non_pow2_no_oob():
    # Reference bug B1/B2: min/max kernel 6 read past the end for non-power-of-2 n. Put a huge
    # sentinel right after the view's end: it must not leak into MAX.
    n = 1_000_001
    base = torch.empty(n + 4096, dtype=torch.float64, device=DEV)
    fill_(base, "uniform", seed=1)
    base[n:] = 1e300
    x = base[:n]
    assert ladder_reduce(x, "max", kernel=6).item() == x.max().item()
    assert reduce(x, "max").item() == x.max().item()


@pytest.mark.parametrize("dt,op,acc", COMBOS, ids=lambda v: str(v).replace("torch.", ""))
@pytest.mark.parametrize("single_pass", [True, False])
def test_bound_reduce_matches_reference(dt, op, acc, single_pass):
    # The prepared launch (_C.BoundReduce) resolves the plan once; launch() may redirect the output.
    n = 3_000_017
    x = torch.empty(n + 1, dtype=dt, device=DEV)[1:]  # misaligned view
    fill_(x, "fullrange" if not dt.is_floating_point else "uniform", seed=41)
    r = Reducer(DEV, config=KernelConfig(single_pass=single_pass))
    out = torch.empty(4, dtype=acc, device=DEV)
    b = r.bind(x, op, acc, out=out[0:1])
    assert b.plan["single_pass"] == single_pass and r.last_plan == b.plan
    stream = torch.cuda.current_stream().cuda_stream
    b.launch(stream)
    for i in (1, 2, 3):
        b.launch(stream, out[i:i + 1].data_ptr())
    torch.cuda.synchronize()
    for i in range(4):
        check(out[i].item(), x, op, acc, n)


def test_bound_reduce_graph_capture_and_replay():
    # Captured launches replay with the self-advancing fan-in epoch: no memset node needed.
    n = 5_000_001
    x = torch.empty(n, dtype=torch.float64, device=DEV)
    fill_(x, "uniform", seed=9)
    r = Reducer(DEV)
    slots = torch.zeros(6, dtype=torch.float64, device=DEV)
    b = r.bind(x, "sum", out=slots[0:1])
    b.launch(torch.cuda.current_stream().cuda_stream)  # warm-up outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(6):
            b.launch(torch.cuda.current_stream().cuda_stream, slots[i:i + 1].data_ptr())
    slots.zero_()
    for _ in range(25):
        g.replay()
    torch.cuda.synchronize()
    for i in range(6):
        check(slots[i].item(), x, "sum", torch.float64, n)


@pytest.mark.parametrize("n_steps,chunk", [(7, 3), (32, 32), (5, 8), (1, 32)])
def test_step_graph_runs_exactly_n_steps(n_steps, chunk):
    from cuda_mpi_reductions_amd.utils.graphs import StepGraph
    counter = torch.zeros(1, dtype=torch.int64, device=DEV)

    def step(j):
        counter.add_(1)
    sg = StepGraph(step, n_steps, torch.device(DEV), chunk=chunk)
    assert sg.capture(), sg.error
    assert sg.captured
    counter.zero_()
    sg.run()
    torch.cuda.synchronize()
    assert counter.item() == n_steps
    assert sg.reps * sg.chunk + sg.rem == n_steps


def test_step_graph_failed_capture_falls_back():
    from cuda_mpi_reductions_amd.utils.graphs import StepGraph

    def bad_step(j):
        torch.cuda.synchronize()  # not allowed while capturing
    sg = StepGraph(bad_step, 4, torch.device(DEV), chunk=2)
    assert not sg.capture() and not sg.captured and sg.error
    # the device is still usable afterwards
    assert torch.ones(3, device=DEV).sum().item() == 3.0


@pytest.mark.parametrize("dt", [torch.int32, torch.int64, torch.float32, torch.float64])
@pytest.mark.parametrize("where", ["first", "last", "random", "tile_edge"])
def test_planted_extremes_large(dt, where):
    # a planted min and max in a large array (no CPU oracle needed) — at the
    # unaligned head, the sub-vector tail, a random index, and the last full-tile boundary.
    import random
    n = 150_000_007
    base = torch.empty(n + 3, dtype=dt, device=DEV)
    x = base[3:]  # misaligned: exercises the scalar head
    fill_(x, "uniform" if dt.is_floating_point else "smallint", seed=77)
    rng = random.Random(hash((str(dt), where)) & 0xFFFF)
    if where == "first":
        i_min, i_max = 0, 1
    elif where == "last":
        i_min, i_max = n - 1, n - 2
    elif where == "tile_edge":
        vec = 16 // x.element_size()
        i_min = (n // (256 * 2 * vec)) * (256 * 2 * vec) - 1
        i_max = i_min + 1
    else:
        i_min, i_max = rng.randrange(n), rng.randrange(n)
        if i_max == i_min:
            i_max = (i_min + 1) % n
    lo, hi = (-1.5, 2.5) if dt.is_floating_point else (-7, 1 << 20)
    x[i_min] = lo
    x[i_max] = hi
    assert reduce(x, "min").item() == lo
    assert reduce(x, "max").item() == hi
    del base, x
    torch.cuda.empty_cache()


# ---- explicit load windows (reduce_kernels.hpp stream_window; round 3, profiles/r3_window)
WINDOWS = [(b, u, w) for b in (256, 512) for u in (2, 4, 8) for w in (2, 4) if u % w == 0]


@pytest.mark.parametrize("block,unroll,window", WINDOWS, ids=lambda v: str(v))
@pytest.mark.parametrize("dt,op,acc", COMBOS, ids=lambda v: str(v).replace("torch.", ""))
@pytest.mark.parametrize("n,misalign", [(5, 0), (1_000_003, 1), (3_000_017, 0)])
def test_window_variants(block, unroll, window, dt, op, acc, n, misalign):
    # every instantiated window against the fp64/int64 reference: tiny n (no full tile: the body is
    # skipped), a misaligned head, and tile counts that do not divide the grid
    base = torch.empty(n + misalign, dtype=dt, device=DEV)
    fill_(base, "fullrange" if not dt.is_floating_point else "uniform", seed=n + 13 * misalign + window)
    x = base[misalign:]
    r = Reducer(DEV, config=KernelConfig(block=block, unroll=unroll, window=window))
    got = r(x, op, acc).item()
    assert r.last_plan["window"] == window and r.last_plan["nontemporal"]
    check(got, x, op, acc, n)


@pytest.mark.parametrize("dt,op", [(torch.bfloat16, "sum"), (torch.float16, "max"), (torch.float64, "sumsq"),
                                   (torch.float32, "amax"), (torch.float32, "sumsq")])
def test_window_fused_and_half_types(dt, op):
    n = 2_000_011
    x = torch.empty(n, dtype=dt, device=DEV)
    fill_(x, "uniform", seed=5)
    r = Reducer(DEV, config=KernelConfig(block=256, unroll=8, window=4))
    got = r(x, op).item()
    xd = x.double()
    ref = {"sum": lambda: xd.sum(), "max": lambda: xd.max(), "sumsq": lambda: (xd * xd).sum(),
           "amax": lambda: xd.abs().max()}[op]().item()
    if op in ("sum", "sumsq"):
        acc = torch.float64 if dt == torch.float64 or (dt == torch.float32 and op == "sumsq") else torch.float32
        tol = sum_tolerance(dt, acc, n, (xd * xd).sum().item() if op == "sumsq" else xd.abs().sum().item())
        assert abs(got - ref) <= tol, (got, ref, tol)
    else:
        assert got == ref
    assert r.last_plan["window"] == 4


@pytest.mark.parametrize("dt,op", [(torch.float64, "sum"), (torch.int64, "min"), (torch.int64, "sum")])
def test_default_plan_above_192mb_uses_the_window(dt, op):
    # the tuned plan for 8-byte arrays > 192 MB is 256x8x1 with window 4: check it at 320 MB, misaligned
    n = 40_000_003
    base = torch.empty(n + 1, dtype=dt, device=DEV)
    fill_(base, "fullrange" if not dt.is_floating_point else "uniform", seed=77)
    x = base[1:]
    r = Reducer(DEV)
    got = r(x, op).item()
    p = r.last_plan
    assert (p["block"], p["unroll"], p["window"]) == (256, 8, 4), p
    check(got, x, op, dt if op != "sum" or dt.is_floating_point else torch.int64, n)


@pytest.mark.parametrize("dt,op,want", [
    (torch.float32, "sum", (256, 8, 1, 4)), (torch.float32, "max", (256, 8, 1, 4)),
    (torch.int32, "max", (256, 8, 1, 4)), (torch.int32, "sum", (256, 8, 2, 2)),
    (torch.bfloat16, "sum", (256, 8, 1, 4)), (torch.float16, "min", (256, 8, 2, 2))])
def test_default_plan_above_192mb_narrow_types(dt, op, want):
    # the round-3 defaults for 4- and 2-byte arrays > 192 MB (profiles/r3_types/): (block, unroll,
    # workgroups per CU, window), misaligned by one element (head scalar + tail), 256 MB of data
    n = (256 << 20) // torch.empty((), dtype=dt).element_size() + 3
    base = torch.empty(n + 1, dtype=dt, device=DEV)
    fill_(base, "fullrange" if not dt.is_floating_point else "uniform", seed=78)
    x = base[1:]
    r = Reducer(DEV)
    got = r(x, op).item()
    p = r.last_plan
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    assert (p["block"], p["unroll"], p["grid"], p["window"]) == (want[0], want[1], cus * want[2], want[3]), p
    half = dt in (torch.bfloat16, torch.float16)
    wide = {torch.int32: torch.int64, torch.float32: torch.float64}
    acc = torch.float32 if half else (wide[dt] if op == "sum" else dt)
    check(got, x, op, acc, n)



@pytest.mark.parametrize("permille", [-300, -16, 0, 9, 16, 400, 5000])
@pytest.mark.parametrize("n", [26_000_003, 31_457_280 + 17])  # 8-byte window plans: > 192 MiB
@pytest.mark.parametrize("op", ["sum", "max"])
def test_xcd_weighted_split(monkeypatch, permille, n, op):
    # round 4: the XCD-weighted split of the window body (reduce_kernels.hpp weighted_tiles) gives
    # one blockIdx parity more rounds; every tile must still be streamed exactly once, for any skew
    # (also skews larger than the array, which leave the other parity without tiles). int64 data:
    # exact SUM / MAX against torch.
    monkeypatch.setenv("MIREDUCE_XCD_SKEW", str(permille))
    C = native()
    g = torch.Generator(device="cpu").manual_seed(n + permille)
    x = torch.randint(-(1 << 40), 1 << 40, (n,), generator=g, dtype=torch.int64).to(DEV)
    if op == "max":
        x[(n * 7) // 11] = 1 << 50  # the extreme sits in one tile
    red = Reducer(torch.device(DEV))
    out = torch.zeros(1, dtype=torch.int64, device=DEV)
    from cuda_mpi_reductions_amd.ops import dtype_code, op_code
    plan = C.reduce(red.ws, x.data_ptr(), n, dtype_code(x.dtype), op_code(op), dtype_code(torch.int64),
                    out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert plan["window"] > 0 and plan["grid"] % 2 == 0, plan
    ntiles = n // 2 // (plan["block"] * plan["unroll"])
    rounds = ntiles // plan["grid"]
    q = rounds * permille + (500 if permille >= 0 else -500)  # the planner's rounding (half away from 0)
    d = (abs(q) // 1000) * (1 if q >= 0 else -1)
    # no skew when it would leave no common round (the kernel anchors the split at their end)
    assert plan["xskew"] == (d if abs(d) * (plan["grid"] // 2) + plan["grid"] <= ntiles else 0), plan
    exp = x.sum().item() if op == "sum" else x.max().item()
    assert out.item() == exp and red.check() is None


def test_reduce_partials_is_unskewed(monkeypatch):
    # reduce_partials has no workspace, so no fan-in epoch to anchor the weighted split with: it
    # streams equal rounds even under an explicit skew, and its partials fold to the exact sum
    monkeypatch.setenv("MIREDUCE_XCD_SKEW", "100")
    n = 26_000_003
    g = torch.Generator(device="cpu").manual_seed(23)
    x = torch.randint(-(1 << 40), 1 << 40, (n,), generator=g, dtype=torch.int64).to(DEV)
    parts, plan = reduce_partials(x, "sum")
    assert plan["window"] > 0 and plan["xskew"] == 0, plan
    assert parts.sum().item() == x.sum().item()


@pytest.mark.parametrize("permille", [100, -100])
@pytest.mark.parametrize("stream", ["current", "side"])
@pytest.mark.parametrize("single_pass", [True, False])
def test_xcd_weighted_split_follows_the_xccs(monkeypatch, permille, stream, single_pass):
    # The weighted split is anchored to the XCDs, not to blockIdx parity (XcdAnchor): which XCD
    # runs workgroup 0 is not fixed (the reduction app's launches were dealt otherwise than
    # tools/xcd_balance.py's, profiles/r4_ab/), so workgroup 0 publishes its XCC's parity and
    # every workgroup derives the favoured blockIdx parity from it. On torch's stream and on a
    # side stream, the workgroups with the extra rounds are exactly
    # those on odd (permille > 0) / even XCCs (the production kernel's own stamps: XCC, tiles), and
    # the sum stays exact — single-pass (polled fan-in epoch) and two-pass (the finalize launch ends
    # the epoch).
    monkeypatch.setenv("MIREDUCE_XCD_SKEW", str(permille))
    C = native()
    n = 26_000_003
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randint(-(1 << 40), 1 << 40, (n,), generator=g, dtype=torch.int64).to(DEV)
    red = Reducer(torch.device(DEV))
    out = torch.zeros(1, dtype=torch.int64, device=DEV)
    st = torch.zeros(3 * red.ws.max_grid, dtype=torch.int64, device=DEV)
    s = torch.cuda.current_stream() if stream == "current" else torch.cuda.Stream()
    from cuda_mpi_reductions_amd.ops import dtype_code, op_code
    torch.cuda.synchronize()
    for k in range(3):  # later launches too: the anchor word carries an earlier launch's tag
        plan = C.reduce(red.ws, x.data_ptr(), n, dtype_code(x.dtype), op_code("sum"), dtype_code(torch.int64),
                        out.data_ptr(), s.cuda_stream, single_pass=single_pass, wg_stamps=st.data_ptr())
        s.synchronize()
        assert plan["single_pass"] == single_pass
        assert out.item() == x.sum().item() and red.check() is None
        assert plan["xskew"] != 0 and plan["xskew"] * permille > 0, plan
        grid = plan["grid"]
        v = st[: 3 * grid].view(grid, 3).cpu()
        odd = v[:, 1] % 2 == 1
        fav, other = (v[odd, 2], v[~odd, 2]) if permille > 0 else (v[~odd, 2], v[odd, 2])
        assert len(fav) == len(other) == grid // 2, (len(fav), len(other))
        assert int(fav.min()) > int(other.max()), (fav.tolist()[:8], other.tolist()[:8])
        assert int(v[:, 2].sum()) == n // 2 // (plan["block"] * plan["unroll"])  # every full tile once


# ---------------------------------------------------------------- segmented launches (round 5)

@pytest.mark.parametrize("dt,op,acc", [(torch.float64, "sum", torch.float64), (torch.float64, "min", torch.float64),
                                       (torch.int64, "sum", torch.int64), (torch.int32, "sum", torch.int64),
                                       (torch.float32, "max", torch.float32), (torch.int64, "max", torch.int64)],
                         ids=lambda v: str(v).replace("torch.", ""))
@pytest.mark.parametrize("misalign", [0, 1])
def test_segmented_launches_match_the_reference(dt, op, acc, misalign):
    # A reduction split into consecutive launches (ReduceConfig::segment_bytes; auto above 16 GiB):
    # every earlier segment's result is carried into the last launch's finisher. Forced here onto a
    # 160-320 MB array in 8 MiB segments (20-39 launches), through reduce() and through a bound launch,
    # on an odd count at an odd offset so segment edges cut vectors and tiles.
    n = 40_000_003
    base = torch.empty(n + misalign, dtype=dt, device=DEV)
    fill_(base, "fullrange" if not dt.is_floating_point else "uniform", seed=91 + misalign)
    x = base[misalign:]
    red = Reducer(DEV, config=KernelConfig(segment_bytes=8 << 20))
    out = red(x, op, acc)
    plan = red.last_plan
    assert plan["segments"] >= 19 and plan["segment_elems"] * plan["segments"] >= n, plan  # 160-320 MB / 8 MiB
    check(out.item(), x, op, acc, n)
    b = red.bind(x, op, acc)
    slot = torch.zeros(4, dtype=acc, device=DEV)
    for i in range(4):  # back-to-back: carried results are rewritten by every launch
        b.launch(torch.cuda.current_stream().cuda_stream, slot[i:i + 1].data_ptr())
    torch.cuda.synchronize()
    assert red.check() is None
    for v in slot.tolist():
        check(v, x, op, acc, n)


def test_segmented_launch_with_fused_finish_world1():
    # the last segment's launch does the fused cross-rank finish (world 1: bound, exchanges nothing)
    from cuda_mpi_reductions_amd.parallel.xrank import close_channels, open_channel
    dev = torch.device(DEV)
    x = torch.empty(30_000_001, dtype=torch.float64, device=dev)
    fill_(x, "uniform", seed=5)
    ch = open_channel(dev, timeout_s=5.0)
    red = Reducer(dev, config=KernelConfig(segment_bytes=16 << 20))
    out = torch.zeros(1, dtype=torch.float64, device=dev)
    b = red.bind(x, "sum", torch.float64, out=out, xrank=ch)
    assert b.plan["segments"] > 10
    for _ in range(3):
        b.launch(torch.cuda.current_stream().cuda_stream, out.data_ptr())
    torch.cuda.synchronize()
    assert int(ch.error()) == 0 and red.check() is None
    check(out.item(), x, "sum", torch.float64, x.numel())
    del b
    close_channels([ch], dev)


def test_segmented_launch_poisons_on_a_late_workgroup():
    # a fan-in failure in any segment poisons the final result (the sticky error word reaches the
    # last segment's finisher) and is reported; the launch after the reset is exact
    C = native()
    from cuda_mpi_reductions_amd.ops import dtype_code, op_code
    dev = torch.device(DEV)
    g = torch.Generator(device="cpu").manual_seed(31)  # (CPU RNG: an earlier graph capture may own the GPU's)
    x = torch.randint(1, 1 << 20, (20_000_000,), generator=g, dtype=torch.int64).to(dev)
    red = Reducer(dev)
    out = torch.zeros(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    plan = C.reduce(red.ws, x.data_ptr(), x.numel(), dtype_code(x.dtype), op_code("sum"), dtype_code(torch.int64),
                    out.data_ptr(), s, segment_bytes=16 << 20, fanin_bound_ticks=100_000, debug_delay_wg=0,
                    debug_delay_ticks=5_000_000)
    torch.cuda.synchronize()
    assert plan["segments"] > 5 and out.item() == 0 and red.ws.error() & 1
    assert red.check() is not None
    C.reduce(red.ws, x.data_ptr(), x.numel(), dtype_code(x.dtype), op_code("sum"), dtype_code(torch.int64),
             out.data_ptr(), s, segment_bytes=16 << 20)
    torch.cuda.synchronize()
    assert red.check() is None and out.item() == x.sum().item()
