"""Fused element-transform operators: SUMSQ (Σ x², the square taken as the element is loaded) and
AMAX (max |x|), for the full reduction, reduce_dim, the host reference and ops.norm (which adds the
reference's scalar cross-rank step: cuda/C/src/simpleMPI/simpleMPI.cpp:92-98). References are plain
PyTorch fp64 reductions of the same tensors."""
import math
import os

import pytest
import torch
import torch.multiprocessing as mp

from cuda_mpi_reductions_amd.ops import (KernelConfig, Reducer, cpu_reduce, default_acc_dtype, fill_, norm, reduce,
                                         reduce_dim, sum_tolerance, synthetic)
from helpers import free_port

FLOATS = [torch.float32, torch.float64, torch.bfloat16, torch.float16]
IDS = ["f32", "f64", "bf16", "f16"]


def _exp(x: torch.Tensor, op: str) -> float:
    xd = x.double()
    return (xd * xd).sum().item() if op == "sumsq" else xd.abs().max().item()


def _check(got: float, x: torch.Tensor, op: str, acc: torch.dtype):
    exp = _exp(x, op)
    if op == "sumsq":
        tol = sum_tolerance(x.dtype, acc, x.numel(), exp)
        # fp32 accumulators also round each square once: allow n * eps32 * Σx² on top
        if acc == torch.float32:
            tol += 6e-8 * exp * 4
        assert abs(got - exp) <= tol, (got, exp, tol)
    else:
        assert got == exp, (got, exp)


def test_accumulators_and_int_rejection():
    assert default_acc_dtype(torch.float32, "sumsq") == torch.float64
    assert default_acc_dtype(torch.float64, "amax") == torch.float64
    assert default_acc_dtype(torch.bfloat16, "sumsq") == torch.float32
    with pytest.raises(TypeError):
        default_acc_dtype(torch.int32, "sumsq")


@pytest.mark.parametrize("dt", FLOATS, ids=IDS)
def test_host_reference(dt):
    x = synthetic(100_003, dt, seed=3)
    x = x * 4 - 2  # signed values: AMAX must take |x|
    acc = default_acc_dtype(dt, "sumsq")
    _check(cpu_reduce(x, "sumsq"), x, "sumsq", acc)
    _check(cpu_reduce(x, "amax"), x, "amax", default_acc_dtype(dt, "amax"))
    r = norm(x)
    assert abs(r.item() - math.sqrt(_exp(x, "sumsq"))) <= 1e-6 * r.item()
    assert norm(x, math.inf).item() == _exp(x, "amax")


def _norm_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    full = synthetic(40_000, torch.float64, seed=17) * 2 - 1
    shard = full.chunk(world)[rank].contiguous()
    q.put((rank, norm(shard).item(), norm(shard, math.inf).item(), norm(full).item(), norm(full, math.inf).item()))
    torch.distributed.destroy_process_group()


def test_distributed_norm_two_ranks():
    """Each rank passes its shard; every rank gets the norm of the whole tensor."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_norm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    full = synthetic(40_000, torch.float64, seed=17) * 2 - 1
    l2, li = torch.linalg.vector_norm(full).item(), full.abs().max().item()
    for _, a, b, _, _ in res:
        assert abs(a - l2) <= 1e-12 * l2 and b == li


# ------------------------------------------------------------------------------------------ GPU
DEV = "cuda:0"


@pytest.mark.gpu
@pytest.mark.parametrize("dt", FLOATS, ids=IDS)
@pytest.mark.parametrize("op", ["sumsq", "amax"])
@pytest.mark.parametrize("n", [1, 3, 64, 1000, 65_537, 1_000_003, (1 << 23) + 9])
@pytest.mark.parametrize("misalign", [0, 1])
def test_gpu_full_reduction(dt, op, n, misalign):
    base = torch.empty(n + misalign, dtype=dt, device=DEV)
    fill_(base, "uniform", seed=n + misalign)
    base.mul_(4).sub_(2)
    x = base[misalign:]
    if op == "amax" and n > 10:
        x[(n * 3) // 5] = -3.75  # the largest magnitude is negative
    acc = default_acc_dtype(dt, op)
    _check(reduce(x, op).item(), x, op, acc)


@pytest.mark.gpu
def test_gpu_fp32_accumulator_and_variants():
    x = synthetic(3_000_017, torch.float32, device=DEV, seed=8) * 3 - 1
    r = Reducer(DEV)
    for block in (256, 512, 1024):
        for unroll in (2, 4, 8, 16):
            cfg = KernelConfig(block=block, unroll=unroll)
            _check(r(x, "sumsq", torch.float32, config=cfg).item(), x, "sumsq", torch.float32)
            _check(r(x, "amax", config=cfg).item(), x, "amax", torch.float32)
    for single_pass in (True, False):
        cfg = KernelConfig(single_pass=single_pass)
        _check(r(x, "sumsq", config=cfg).item(), x, "sumsq", torch.float64)
        _check(r(x, "amax", config=cfg).item(), x, "amax", torch.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", FLOATS, ids=IDS)
def test_gpu_reduce_dim(dt):
    x = synthetic(3000 * 257, dt, device=DEV, seed=2).view(3000, 257) * 2 - 1
    for dim in (0, 1):
        s = reduce_dim(x, "sumsq", dim)
        exp = (x.double() ** 2).sum(dim)
        assert torch.allclose(s.double(), exp, rtol=1e-5 if s.dtype == torch.float32 else 1e-12)
        m = reduce_dim(x, "amax", dim)
        assert torch.equal(m.double(), x.double().abs().amax(dim))


@pytest.mark.gpu
def test_gpu_norm_matches_torch_and_ignores_nan_in_amax():
    x = synthetic(10_000_019, torch.float32, device=DEV, seed=4) * 2 - 1
    assert abs(norm(x).item() - torch.linalg.vector_norm(x.double()).item()) <= 1e-9 * norm(x).item()
    assert norm(x, math.inf).item() == x.abs().max().item()
    x[123] = float("nan")
    assert norm(x, math.inf).item() == x.nan_to_num(0.0).abs().max().item()  # maxNum semantics


@pytest.mark.gpu
@pytest.mark.parametrize("method,ty", [("SUMSQ", "double"), ("SUMSQ", "float"), ("AMAX", "bf16"), ("AMAX", "half")])
def test_gpu_reduction_app(method, ty):
    from helpers import BIN, ensure_built, run
    ensure_built()
    r = run([os.path.join(BIN, "reduction"), f"--method={method}", f"--type={ty}", "--n=16777221",
             "--pattern=uniform", "--iterations=5", "--qatest"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "&&&& PASSED" in r.stdout + r.stderr
