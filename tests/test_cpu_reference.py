"""Host reference reducers (csrc/runtime/cpu_reference.cpp) vs Python / numpy oracles."""
import math
import random

import numpy as np
import pytest
import torch

from cuda_mpi_reductions_amd._native import native
from cuda_mpi_reductions_amd.ops import cpu_reduce, default_acc_dtype, fill_, reduce, sum_tolerance

COMBOS = [
    (torch.int32, "sum", torch.int64), (torch.int32, "sum", torch.int32), (torch.int32, "min", torch.int32),
    (torch.int32, "max", torch.int32), (torch.int64, "sum", torch.int64), (torch.int64, "min", torch.int64),
    (torch.int64, "max", torch.int64), (torch.float32, "sum", torch.float64), (torch.float32, "sum", torch.float32),
    (torch.float32, "min", torch.float32), (torch.float32, "max", torch.float32),
    (torch.float64, "sum", torch.float64), (torch.float64, "min", torch.float64), (torch.float64, "max", torch.float64),
]


def py_expected(vals, op, acc):
    if op == "min":
        return min(vals)
    if op == "max":
        return max(vals)
    if acc.is_floating_point:
        return math.fsum(vals)
    bits = 32 if acc == torch.int32 else 64
    s = sum(vals) % (1 << bits)
    return s - (1 << bits) if s >= (1 << (bits - 1)) else s


@pytest.mark.parametrize("dt,op,acc", COMBOS, ids=lambda v: str(v).replace("torch.", ""))
@pytest.mark.parametrize("n", [1, 2, 17, 1000, 100_003])
def test_cpu_reduce_all_combos(dt, op, acc, n):
    x = torch.empty(n, dtype=dt)
    fill_(x, "fullrange" if not dt.is_floating_point else "uniform", seed=n)
    got = cpu_reduce(x, op, acc)
    exp = py_expected(x.tolist(), op, acc)
    if op == "sum" and acc.is_floating_point:
        tol = sum_tolerance(dt, acc, n, float(x.double().abs().sum()))
        assert abs(got - exp) <= tol
    else:
        assert got == exp


def test_default_accumulators():
    assert default_acc_dtype(torch.int32, "sum") == torch.int64
    assert default_acc_dtype(torch.float32, "sum") == torch.float64
    assert default_acc_dtype(torch.int32, "max") == torch.int32
    assert default_acc_dtype(torch.float64, "min") == torch.float64
    C = native()
    assert not C.acc_supported(0, 1, 1)  # int32 MIN with int64 acc is not a supported combination


def test_compensated_sum_is_accurate():
    # 1e6 x 0.1 + large/small mix: Kahan/Neumaier keeps the error at a few ulp of the result.
    rng = random.Random(5)
    vals = [rng.uniform(-1, 1) * 10 ** rng.randint(-8, 8) for _ in range(200_000)]
    x = torch.tensor(vals, dtype=torch.float64)
    got = cpu_reduce(x, "sum")
    exp = math.fsum(vals)
    assert abs(got - exp) <= 8 * np.spacing(abs(exp))


def test_multithreaded_matches_single_thread_exactly_for_ints():
    C = native()
    x = torch.empty(5_000_011, dtype=torch.int64)
    fill_(x, "fullrange", seed=9)
    a = C.cpu_reduce(x.data_ptr(), x.numel(), 1, 0, 1, 1)
    b = C.cpu_reduce(x.data_ptr(), x.numel(), 1, 0, 1, 8)
    assert a == b == py_expected(x.tolist(), "sum", torch.int64)


def test_host_tensor_reduce_returns_tensor():
    x = torch.arange(10, dtype=torch.int32)
    r = reduce(x, "sum")
    assert r.dtype == torch.int64 and r.item() == 45
    assert reduce(x, "min").item() == 0 and reduce(x, "max").item() == 9


def test_nan_semantics_host():
    x = torch.tensor([1.0, float("nan"), -3.0], dtype=torch.float64)
    assert cpu_reduce(x, "min") == -3.0 and cpu_reduce(x, "max") == 1.0
    assert math.isnan(cpu_reduce(x, "sum"))


def test_empty_identity_host():
    x = torch.empty(0, dtype=torch.float64)
    assert cpu_reduce(x, "sum") == 0.0
    assert cpu_reduce(x, "min") == math.inf and cpu_reduce(x, "max") == -math.inf
    xi = torch.empty(0, dtype=torch.int32)
    assert cpu_reduce(xi, "min") == 2**31 - 1 and cpu_reduce(xi, "max") == -2**31


def test_tolerance_policy():
    C = native()
    assert C.sum_tolerance(0, 1, 100, 1e9) == 0.0       # integer: exact
    t64 = C.sum_tolerance(3, 3, 10**9, 5e8)
    assert 1e-12 <= t64 < 1e-3                          # fp64: tiny relative bound
    t32 = C.sum_tolerance(2, 2, 1000, 500.0)
    assert t32 >= 1e-8 * 1000                           # fp32 acc: at least the reference's 1e-8*n
