"""reduce_dim (csrc/kernels/reduce_dim.hip): per-row / per-column reductions against plain PyTorch
fp64 / int64 references of the same tensors. Shapes cover short rows packed several to a wave,
long rows split into segments (per-row tickets), misaligned bases and odd lengths (scalar head /
tail), column slabs with few columns (row groups + LDS fold) and many rows (split + fold launch),
middle axes of 3-D tensors, every dtype / op / accumulator."""
import math

import pytest
import torch

from cuda_mpi_reductions_amd.ops import fill_, reduce_dim

COMBOS = [
    (torch.float64, "sum", None), (torch.float64, "min", None), (torch.float64, "max", None),
    (torch.float32, "sum", None), (torch.float32, "sum", torch.float32), (torch.float32, "max", None),
    (torch.int32, "sum", None), (torch.int32, "sum", torch.int32), (torch.int32, "min", None),
    (torch.int64, "sum", None), (torch.int64, "max", None),
    (torch.bfloat16, "sum", None), (torch.bfloat16, "min", None),
    (torch.float16, "sum", None), (torch.float16, "max", None),
]
IDS = [f"{str(d).replace('torch.', '')}-{o}-{str(a).replace('torch.', '') if a else 'acc'}" for d, o, a in COMBOS]


def _ref(x: torch.Tensor, op: str, dim: int, acc: torch.dtype):
    if op == "sum":
        if acc.is_floating_point:
            return x.double().sum(dim)
        if acc == torch.int32:
            s = x.long().sum(dim)
            return ((s + 2 ** 31) % 2 ** 32) - 2 ** 31
        return x.long().sum(dim)
    r = x.amin(dim) if op == "min" else x.amax(dim)
    return r.double() if acc.is_floating_point else r.long()


def _check(got: torch.Tensor, x: torch.Tensor, op: str, dim: int):
    exp = _ref(x, op, dim, got.dtype)
    assert got.shape == exp.shape, (got.shape, exp.shape)
    if op == "sum" and got.dtype.is_floating_point:
        # sum_tolerance() of the full reduction, per output element
        n = x.shape[dim]
        eps = 1.1102230246251565e-16 if got.dtype == torch.float64 else 5.960464477539063e-8
        absum = x.double().abs().sum(dim).cpu()
        floor = 1e-8 * n if (x.dtype == torch.float32 and got.dtype == torch.float32) else 1e-12
        tol = torch.clamp((4096.0 + 4.0 * math.log2(n + 2.0)) * eps * absum, min=floor)
        assert ((got.double().cpu() - exp.cpu()).abs() <= tol).all(), (got, exp)
    else:
        assert torch.equal(got.cpu().to(exp.dtype), exp.cpu()), (got, exp)


def test_host_fallback_matches_torch():
    x = torch.randn(6, 9, 5, dtype=torch.float64)
    for dim in range(3):
        assert torch.allclose(reduce_dim(x, "sum", dim), x.sum(dim))
        assert torch.equal(reduce_dim(x, "max", dim, keepdim=True), x.amax(dim, keepdim=True))
    xi = torch.arange(24, dtype=torch.int32).reshape(4, 6)
    assert reduce_dim(xi, "sum", 1).dtype == torch.int64


def _make(shape, dt, misalign=0, seed=1):
    n = math.prod(shape)
    base = torch.empty(n + misalign, dtype=dt, device="cuda")
    fill_(base, "uniform" if dt.is_floating_point else "fullrange", seed=seed)
    if dt in (torch.int32, torch.int64):
        base.remainder_(1 << 20)  # keep int32 sums in range for the int32-accumulator case
    return base[misalign:].view(shape)


@pytest.mark.gpu
@pytest.mark.parametrize("dt,op,acc", COMBOS, ids=IDS)
@pytest.mark.parametrize("shape", [(1, 1), (3, 5), (7, 64), (33, 257), (1000, 3), (129, 1000), (2, 100_003),
                                   (5, 1_000_000), (1, 4_000_037), (100_000, 17)])
@pytest.mark.parametrize("misalign", [0, 1])
def test_rows(dt, op, acc, shape, misalign):
    x = _make(shape, dt, misalign, seed=shape[0] * 7 + shape[1])
    _check(reduce_dim(x, op, -1, acc), x, op, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("dt,op,acc", COMBOS, ids=IDS)
@pytest.mark.parametrize("shape", [(1, 1), (5, 3), (64, 7), (257, 33), (3, 1000), (1000, 129), (100_003, 2),
                                   (1_000_000, 5), (4_000_037, 1), (17, 100_000), (4096, 4096)])
@pytest.mark.parametrize("misalign", [0, 1])
def test_cols(dt, op, acc, shape, misalign):
    x = _make(shape, dt, misalign, seed=shape[0] + shape[1] * 3)
    _check(reduce_dim(x, op, 0, acc), x, op, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float64, torch.bfloat16, torch.int32])
@pytest.mark.parametrize("shape,dim", [((4, 1000, 6), 1), ((70_000, 3, 8), 1), ((3, 5, 7, 9), 2), ((2, 3, 4), 0),
                                       ((8, 16, 4), 2)])
def test_middle_axes(dt, shape, dim):
    x = _make(shape, dt, seed=sum(shape))
    for op in ("sum", "max"):
        _check(reduce_dim(x, op, dim), x, op, dim)


@pytest.mark.gpu
def test_split_rows_are_deterministic_and_reusable():
    """Split rows (per-row tickets) give bit-identical results across repeated launches (the
    tickets are reset by each row's last segment) and match the unsplit full reduction."""
    x = _make((3, 20_000_000), torch.float64, seed=5)
    first = reduce_dim(x, "sum", 1)
    for _ in range(20):
        assert torch.equal(reduce_dim(x, "sum", 1), first)
    _check(first, x, "sum", 1)


@pytest.mark.gpu
def test_nan_and_keepdim_and_out():
    x = torch.zeros(4, 1000, dtype=torch.float32, device="cuda")
    x[2, 500] = float("nan")
    x[1, 10] = 3.0
    m = reduce_dim(x, "max", 1, keepdim=True)
    assert m.shape == (4, 1) and m[1, 0].item() == 3.0 and m[2, 0].item() == 0.0  # maxNum ignores NaN
    s = reduce_dim(x, "sum", 1)
    assert math.isnan(s[2].item()) and s[1].item() == 3.0
    out = torch.empty(1000, dtype=torch.float64, device="cuda")
    assert reduce_dim(x, "sum", 0, out=out) is out
