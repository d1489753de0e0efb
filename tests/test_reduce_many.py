"""reduce_many / ReduceMany / norm_many (csrc/kernels/reduce_many.hip): one launch over a list of
tensors, against per-tensor PyTorch fp64 references. Lists mix empty, tiny, misaligned and
multi-segment tensors; bound lists are relaunched (ticket reset) and captured into a graph."""
import math

import pytest
import torch

from cuda_mpi_reductions_amd.ops import ReduceMany, fill_, norm_many, reduce_many, synthetic


def _ref(t: torch.Tensor, op: str) -> float:
    d = t.double()
    if op == "sum":
        return d.sum().item()
    if op == "sumsq":
        return (d * d).sum().item()
    if op == "amax":
        return d.abs().max().item() if t.numel() else 0.0
    if t.numel() == 0:
        return math.inf if op == "min" else -math.inf
    return (d.min() if op == "min" else d.max()).item()


def _close(got: float, exp: float, op: str, acc: torch.dtype, scale: float):
    if op in ("sum", "sumsq"):
        rel = 1e-5 if acc == torch.float32 else 1e-11
        assert abs(got - exp) <= rel * max(scale, 1e-30) + 1e-12, (got, exp)
    else:
        assert got == exp, (got, exp)


def test_host_lists_fall_back():
    ts = [torch.arange(10, dtype=torch.float64), torch.ones(7, dtype=torch.float64)]
    assert reduce_many(ts, "sum").tolist() == [45.0, 7.0]
    total, per = norm_many(ts)
    assert abs(total.item() - math.sqrt(285 + 7)) < 1e-12 and per.shape == (2,)


def _mixed_list(dt, seed=0):
    sizes = [0, 1, 5, 63, 1000, 4097, 65_536, 1_000_003, 3_000_017, 17]
    base = torch.empty(sum(sizes) + 2 * len(sizes), dtype=dt, device="cuda")
    fill_(base, "uniform", seed=seed)
    base.mul_(2).sub_(1)
    ts, off = [], 0
    for i, n in enumerate(sizes):
        off += i % 3  # misaligned starts
        ts.append(base[off:off + n])
        off += n
    return ts


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float64, torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("op", ["sum", "min", "max", "sumsq", "amax"])
def test_mixed_list(dt, op):
    ts = _mixed_list(dt, seed=3)
    out = reduce_many(ts, op)
    for t, g in zip(ts, out.tolist()):
        exp = _ref(t, op)
        _close(g, exp, op, out.dtype, t.double().abs().sum().item() if op == "sum" else abs(exp))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.int32, torch.int64])
def test_int_lists(dt):
    ts = [synthetic(n, dt, device="cuda", pattern="fullrange", seed=n) for n in (1, 100, 200_003, 5_000_011)]
    for op in ("sum", "min", "max"):
        out = reduce_many(ts, op)
        for t, g in zip(ts, out.tolist()):
            exp = t.long().sum().item() if op == "sum" else (t.min() if op == "min" else t.max()).item()
            assert g == exp


@pytest.mark.gpu
def test_many_small_tensors_one_launch():
    ts = [synthetic(n, torch.float32, device="cuda", seed=n) for n in range(1, 1001)]
    rm = ReduceMany(ts, "sumsq")
    out = rm().tolist()
    for t, g in zip(ts, out):
        assert abs(g - (t.double() ** 2).sum().item()) <= 1e-9 * max(1.0, g)


@pytest.mark.gpu
def test_bound_relaunch_and_graph_capture():
    ts = _mixed_list(torch.float64, seed=9)
    rm = ReduceMany(ts, "sum")
    first = rm().clone()
    for _ in range(30):  # tickets must be left at zero by every launch
        assert torch.equal(rm(), first)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            rm(s)
    rm.out.zero_()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(rm.out, first)


@pytest.mark.gpu
def test_reduce_many_caches_the_binding_and_returns_fresh_tensors():
    # repeated calls on the same list reuse one binding (no per-call allocation,
    # upload or sync) and every call returns its own result tensor.
    import importlib
    from cuda_mpi_reductions_amd.ops import reduce_many as rmod
    m = importlib.import_module("cuda_mpi_reductions_amd.ops.reduce_many")  # (the package re-exports the function)
    ts = _mixed_list(torch.float32, seed=3)
    m._bindings.clear()
    a = rmod(ts, "sum")
    b = rmod(ts, "sum")
    assert len(m._bindings) == 1 and a.data_ptr() != b.data_ptr()
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    ref = torch.stack([t.double().sum() for t in ts])
    assert torch.allclose(a, ref, rtol=1e-9, atol=1e-9)
    ts[0].add_(1.0)  # same storage, new values: the cached binding reads them
    c = rmod(ts, "sum")
    assert abs(c[0].item() - (a[0].item() + ts[0].numel())) <= 1e-6 * max(1.0, abs(c[0].item()))


@pytest.mark.gpu
def test_reduce_inside_capture_without_reducer_raises_clearly(monkeypatch):
    # (simulated capture: raising inside a real torch.cuda.graph context leaves torch's graph state
    # unregistered and aborts the process at exit in this torch build)
    from cuda_mpi_reductions_amd.ops import reduce
    x = torch.ones(1000, dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()  # a stream with no reducer yet
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    with torch.cuda.stream(s):
        with pytest.raises(RuntimeError, match="inside a hipGraph capture"):
            reduce(x)
    monkeypatch.undo()
    with torch.cuda.stream(s):
        assert reduce(x).item() == 1000.0


@pytest.mark.gpu
def test_norm_many_matches_torch():
    ts = _mixed_list(torch.float32, seed=5)
    total, per = norm_many(ts)
    ref = torch.linalg.vector_norm(torch.cat([t.double() for t in ts])).item()
    assert abs(total.item() - ref) <= 1e-9 * ref
    tot_inf, _ = norm_many(ts, math.inf)
    assert tot_inf.item() == max(t.abs().max().item() for t in ts if t.numel())
