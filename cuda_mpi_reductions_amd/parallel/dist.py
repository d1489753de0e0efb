"""Process-group setup, sharding and cross-rank reductions over ``torch.distributed``.

One process per GPU; on ROCm the "nccl" backend IS RCCL, whose collectives run over the xGMI
links of an MI355X node. On hosts without a GPU the same code runs over gloo (tests).

Reference parity:
* ``MPI_Init`` / ``MPI_Comm_rank`` / ``MPI_Comm_size`` (mpi/reduce.c:32-34) -> :func:`init`
* the ``N/P`` per-rank split (mpi/reduce.c:43-44) -> :func:`shard` (remainder distributed instead
  of dropped, bug B10)
* element-wise vector ``MPI_Reduce`` to root 0 (mpi/reduce.c:62-63,76,90) -> :func:`vector_reduce`
* the hybrid local-reduce + scalar ``MPI_Reduce`` of the vendored simpleMPI
  (cuda/C/src/simpleMPI/simpleMPI.cpp:92-98) -> :func:`scalar_allreduce`
"""
from __future__ import annotations

import contextlib
import datetime
import os
import socket
import sys
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

__all__ = ["DistContext", "init", "shutdown", "shard", "reduce_op", "scalar_allreduce",
           "vector_reduce", "vector_allreduce", "loc_allreduce", "barrier", "max_over_ranks", "agree",
           "PeerLost"]

# The fused ops exchange already-transformed partials (sum of x^2, max |x|) and combine them
# like SUM / MAX across ranks.
_REDUCE_OPS = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX,
               "sumsq": dist.ReduceOp.SUM, "amax": dist.ReduceOp.MAX}


def reduce_op(op: str):
    try:
        return _REDUCE_OPS[op.lower()]
    except KeyError:
        raise ValueError(f"unsupported op {op!r}") from None


@dataclass
class DistContext:
    rank: int
    world_size: int
    local_rank: int
    backend: str
    device: torch.device
    owns_group: bool

    @property
    def is_root(self) -> bool:
        return self.rank == 0


@contextlib.contextmanager
def stdout_to_stderr():
    """Route fd 1 to stderr: RCCL prints a version banner on stdout when a communicator is
    created, and stdout of our tools carries data (JSON / GNUPlot lines)."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def init(backend: Optional[str] = None, device_type: Optional[str] = None,
         timeout_s: float = 600.0) -> DistContext:
    """Initialise (or join) the default process group from torchrun-style env variables.

    Without RANK/WORLD_SIZE in the environment a 1-rank group is created on 127.0.0.1 so
    single-GPU runs go through exactly the same code path as multi-GPU ones.
    """
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if backend is None:
        backend = "nccl" if device_type == "cuda" else "gloo"
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device_type == "cuda":
        # MIREDUCE_FORCE_DEVICE pins every rank to one GPU: a rehearsal of the multi-rank GPU path
        # on a 1-GPU box (with backend gloo — RCCL refuses two ranks on one device).
        dev_index = int(os.environ.get("MIREDUCE_FORCE_DEVICE", local_rank))
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    owns = False
    if not dist.is_initialized():
        kwargs = dict(backend=backend, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if world == 1 and "MASTER_PORT" not in os.environ:
            # A lone process (not launched by torchrun): an in-process store, no TCP rendezvous —
            # picking a free port and binding it again later can lose the port to another process
            # in between (EADDRINUSE seen on the GPU box).
            kwargs["store"] = dist.HashStore()
        else:
            if "MASTER_ADDR" not in os.environ:
                os.environ["MASTER_ADDR"] = "127.0.0.1"
            if "MASTER_PORT" not in os.environ:
                os.environ["MASTER_PORT"] = str(_free_port())
        if backend == "nccl":
            kwargs["device_id"] = device  # eager communicator creation, inside the redirect
        with stdout_to_stderr():
            dist.init_process_group(**kwargs)
            if backend == "nccl":
                dist.barrier(device_ids=[device.index])
        owns = True
    return DistContext(rank, world, local_rank, backend, device, owns)


def shutdown(ctx: Optional[DistContext] = None) -> None:
    if dist.is_initialized() and (ctx is None or ctx.owns_group):
        from .topology import forget
        forget()  # answers remembered per process group go with the groups
        dist.destroy_process_group()


def shard(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """(offset, count) of this rank's contiguous shard; the first ``n % world`` ranks get one
    extra element so the shards cover all ``n_total`` elements."""
    base, rem = divmod(n_total, world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def barrier(ctx: DistContext) -> None:
    if ctx.world_size > 1 or dist.is_initialized():
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()


def scalar_allreduce(t: torch.Tensor, op: str = "sum", async_op: bool = False):
    """Cross-rank all-reduce of a (1-element) local result, in place."""
    return dist.all_reduce(t, op=reduce_op(op), async_op=async_op)


def vector_allreduce(t: torch.Tensor, op: str = "sum", async_op: bool = False):
    """Element-wise all-reduce of an N/P vector (every rank gets the result)."""
    return dist.all_reduce(t, op=reduce_op(op), async_op=async_op)


def vector_reduce(t: torch.Tensor, op: str = "sum", root: int = 0, async_op: bool = False):
    """Element-wise reduce to ``root`` — the ``MPI_Reduce`` of mpi/reduce.c:76,90."""
    return dist.reduce(t, dst=root, op=reduce_op(op), async_op=async_op)


def loc_allreduce(value: torch.Tensor, index: torch.Tensor, op: str = "max", group=None):
    """``MPI_MAXLOC`` / ``MPI_MINLOC`` of one (value, global index) pair per rank: every rank gets
    the extreme value and, among the ranks holding it, the smallest index (NaN is the extreme, as
    in :func:`ops.arg_reduce`). Two 1-element all-gathers, then a device-side pick — no host
    synchronisation, so it can be captured into a hipGraph with the local arg-reduction."""
    if op not in ("max", "min"):
        raise ValueError("loc_allreduce: op must be 'max' or 'min'")
    world = dist.get_world_size(group)
    v = value.reshape(1)
    i = index.reshape(1).to(torch.int64)
    if dist.get_backend(group) == "gloo" and v.device.type != "cpu":
        hv, hi = loc_allreduce(v.cpu(), i.cpu(), op, group)
        return hv.to(v.device), hi.to(v.device)
    vals = torch.empty(world, dtype=v.dtype, device=v.device)
    idxs = torch.empty(world, dtype=torch.int64, device=v.device)
    if dist.get_backend(group) == "gloo":
        dist.all_gather(list(vals.chunk(world)), v, group=group)
        dist.all_gather(list(idxs.chunk(world)), i, group=group)
    else:
        dist.all_gather_into_tensor(vals, v, group=group)
        dist.all_gather_into_tensor(idxs, i, group=group)
    best = vals.amax() if op == "max" else vals.amin()  # torch propagates NaN, like arg_reduce
    same = vals == best
    if vals.is_floating_point():
        same = same | (torch.isnan(vals) & torch.isnan(best))
    cand = torch.where(same, idxs, torch.full_like(idxs, torch.iinfo(torch.int64).max))
    return best.reshape(1), cand.min().reshape(1)


def max_over_ranks(value: float, ctx: DistContext) -> float:
    """MAX of a host float over all ranks (timing: the slowest rank defines the step)."""
    if ctx.world_size == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64,
                     device=ctx.device if ctx.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class PeerLost(RuntimeError):
    """A bounded agreement (:func:`agree`) ended without every rank's report: the ``missing``
    ranks died or hang, so no collective of the job can complete any more."""

    def __init__(self, stage: str, missing: list, timeout_s: float):
        self.stage, self.missing, self.timeout_s = stage, list(missing), timeout_s
        who = ", ".join(str(r) for r in self.missing)
        super().__init__(f"{stage}: rank(s) {who} did not report within {timeout_s:g} s (dead or hung)")


_agree_seq = [0]


def _store():
    from torch.distributed import distributed_c10d as c10d
    return c10d._get_default_store()


def agree(ctx: DistContext, stage: str, payload: dict, timeout_s: float = 60.0) -> list:
    """Every rank's ``payload`` (JSON-serialisable), in rank order, exchanged through the job's
    rendezvous store instead of a process-group collective — so the wait is BOUNDED: a rank that
    died or hangs is detected after ``timeout_s`` (:class:`PeerLost` names it) rather than waited on
    until the process-group timeout, and a rank whose part of a stage raised still reports (its
    payload carries the error). Every rank must call it the same number of times in the same order
    (the keys carry a per-process sequence number). Used by bench.py's optional headline stages
    (canary verdicts, the fused self-check, plan tuning), whose failure on any rank must turn into
    an agreed fallback, not a hang (the reference ends every job by its wall
    time, mpi/submit_all.sh:4)."""
    import json
    if ctx.world_size == 1 or not dist.is_initialized():
        return [payload]
    _agree_seq[0] += 1
    base = f"mireduce/agree/{_agree_seq[0]}/{stage}/"
    store = _store()
    store.set(base + str(ctx.rank), json.dumps(payload))
    keys = [base + str(r) for r in range(ctx.world_size)]
    try:
        store.wait(keys, datetime.timedelta(seconds=max(0.1, timeout_s)))
    except Exception:  # noqa: BLE001 - a store timeout (DistStoreError / RuntimeError): find who is missing
        missing = []
        for r, k in enumerate(keys):
            if r == ctx.rank:
                continue  # (this rank's own report was set above)
            try:
                if not store.check([k]):
                    missing.append(r)
            except Exception:  # noqa: BLE001 - the store itself is gone (its host, rank 0, died)
                missing.append(r)
        if missing:
            raise PeerLost(stage, missing, timeout_s) from None
    return [json.loads(store.get(k)) for k in keys]
