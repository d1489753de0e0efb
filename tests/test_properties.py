"""Property-based tests (hypothesis) of the host-side contracts every GPU path relies on.

* counter-based data: element i = f(seed, i), so any chunking/sharding of the fill gives the same
  logical array (what lets bench.py shard 1e9 elements over 1..8 ranks and still verify);
* the native host reducers equal exact / fp64 references for every (dtype, op, accumulator)
  (the CPU oracle of reduction.cpp:748-780, here with wrap semantics and 64-bit sizes);
* sharding covers [0, n) exactly (the N/P split of mpi/reduce.c:43-44 without dropping the
  remainder, bug B10);
* output lines round-trip through the parsers getAvgs / plotting use (reduce.c:68,81,95;
  reduction.cpp:744-745);
* the fault-spec grammar round-trips.
"""
import math

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from cuda_mpi_reductions_amd.ops import cpu_reduce, synthetic
from cuda_mpi_reductions_amd.parallel.dist import shard
from cuda_mpi_reductions_amd.utils.fault import FaultSpec, parse_fault_spec
from cuda_mpi_reductions_amd.utils.formats import gnuplot_line, parse_gnuplot, parse_throughput, throughput_line

SETTINGS = settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
DTYPES = [torch.int32, torch.int64, torch.float32, torch.float64]
PATTERNS = ["uniform", "smallint", "fullrange", "iotamod", "constant"]


@SETTINGS
@given(n=st.integers(1, 5000), cut=st.integers(0, 5000), seed=st.integers(0, 2**63 - 1),
       dt=st.sampled_from(DTYPES), pattern=st.sampled_from(PATTERNS))
def test_fill_is_chunking_invariant(n, cut, seed, dt, pattern):
    cut = min(cut, n)
    whole = synthetic(n, dt, pattern=pattern, seed=seed, value=3.0)
    a = synthetic(cut, dt, pattern=pattern, seed=seed, value=3.0)
    b = synthetic(n - cut, dt, pattern=pattern, seed=seed, offset=cut, value=3.0)
    assert torch.equal(whole, torch.cat([a, b]))


@SETTINGS
@given(n=st.integers(0, 1 << 40), world=st.integers(1, 1024))
def test_shard_partitions_exactly(n, world):
    parts = [shard(n, r, world) for r in range(min(world, 8))] + [shard(n, world - 1, world)]
    assert parts[0][0] == 0
    for (o1, c1), (o2, _) in zip(parts[:-2], parts[1:-1]):
        assert o1 + c1 == o2
    last_off, last_cnt = parts[-1]
    assert last_off + last_cnt == n
    base = n // world
    assert all(c in (base, base + 1) for _, c in parts)


def _int_ref(x: np.ndarray, op: str, bits: int) -> int:
    if op == "min":
        return int(x.min())
    if op == "max":
        return int(x.max())
    s = int(x.astype(object).sum())
    m = 1 << bits
    s %= m
    return s - m if s >= m // 2 else s


@SETTINGS
@given(data=st.data(), dt=st.sampled_from(DTYPES), op=st.sampled_from(["sum", "min", "max"]))
def test_cpu_reduce_matches_reference(data, dt, op):
    n = data.draw(st.integers(1, 3000))
    seed = data.draw(st.integers(0, 2**32))
    x = synthetic(n, dt, pattern="fullrange" if not dt.is_floating_point else "uniform", seed=seed)
    got = cpu_reduce(x, op)
    xn = x.numpy()
    if dt.is_floating_point:
        if op == "sum":
            ref = math.fsum(float(v) for v in xn)
            assert abs(got - ref) <= 1e-12 * max(1.0, abs(ref)) * (1 if dt == torch.float64 else 1e4)
        else:
            assert got == float(xn.min() if op == "min" else xn.max())
    else:
        # int32 SUM accumulates in int64 by default (no wrap); everything else keeps its width
        bits = 64 if (dt == torch.int64 or op == "sum") else 32
        assert got == _int_ref(xn, op, bits)


@SETTINGS
@given(n=st.integers(1, 3000), seed=st.integers(0, 2**32))
def test_cpu_reduce_int32_acc_wraps_like_mpi_int(n, seed):
    x = synthetic(n, torch.int32, pattern="fullrange", seed=seed)
    assert cpu_reduce(x, "sum", torch.int32) == _int_ref(x.numpy(), "sum", 32)


@SETTINGS
@given(dtype=st.sampled_from(["INT", "DOUBLE", "LONG", "FLOAT"]), op=st.sampled_from(["MAX", "MIN", "SUM"]),
       nodes=st.integers(1, 1 << 20), v=st.floats(0, 1e7, allow_nan=False))
def test_gnuplot_line_round_trip(dtype, op, nodes, v):
    line = gnuplot_line(dtype, op, nodes, v)
    (row,) = list(parse_gnuplot([line]))
    assert (row.dtype, row.op, row.nodes) == (dtype, op, nodes)
    assert abs(row.value - v) <= 5e-4 + 1e-12 * v


@SETTINGS
@given(gbs=st.floats(0, 1e5, allow_nan=False), secs=st.floats(0, 100, allow_nan=False),
       n=st.integers(0, 1 << 40), devs=st.integers(1, 8), wg=st.sampled_from([64, 256, 512, 1024]))
def test_throughput_line_round_trip(gbs, secs, n, devs, wg):
    d = parse_throughput(throughput_line(gbs, secs, n, devs, wg))
    assert d["elements"] == n and d["num_devs"] == devs and d["workgroup"] == wg
    assert abs(d["gb_per_s"] - gbs) <= 5e-5 + 1e-12 * gbs and abs(d["seconds"] - secs) <= 5e-6 + 1e-12 * secs


@SETTINGS
@given(kind=st.sampled_from(["exit", "hang", "corrupt", "delay"]), rank=st.one_of(st.none(), st.integers(0, 4096)),
       step=st.one_of(st.none(), st.integers(0, 10**9)), ms=st.integers(0, 10**6))
def test_fault_spec_round_trip(kind, rank, step, ms):
    spec = (f"delay={ms}" if kind == "delay" else kind) + ("" if rank is None else f"@{rank}") + \
        ("" if step is None else f":{step}")
    f = parse_fault_spec(spec)
    assert f == FaultSpec(kind, 1 if rank is None else rank, 0 if step is None else step, ms if kind == "delay" else 0)


@pytest.mark.parametrize("spec", ["", "none"])
def test_fault_spec_none(spec):
    assert parse_fault_spec(spec).kind == "none"
