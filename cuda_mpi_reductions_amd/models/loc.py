"""MAXLOC / MINLOC workload: the position of the global extreme of a sharded array.

MPI's location reductions (``MPI_MAXLOC`` / ``MPI_MINLOC``) are the standard companions of the
MAX / MIN that mpi/reduce.c times (mpi/reduce.c:21-28,76,90); the reference's CUDA side returns
extreme values only (cuda/C/src/reduction/reduction_kernel.cu:128-253). A step here is the
north-star shape — local HIP pass over this rank's shard, then a tiny cross-rank combine:

* local: ``arg_reduce_rows`` (csrc/kernels/arg_reduce.hip) on a prepared scratch buffer — first
  index of the extreme and its value, one launch, single-pass finish;
* global, GPUs over RCCL: ``loc_pack`` writes this rank's (value key, global index) pair, ONE
  all-gather of the pairs, ``loc_pick`` folds them with arg_reduce's rules and writes the global
  index into the step's slot — three launches and one collective per step (the torch version, two
  all-gathers and ~8 elementwise ops, cost 27 us per step at N=1: profiles/r3_configs/);
* global, gloo / CPU ranks: :func:`parallel.dist.loc_allreduce` (two all-gathers and a pick).

No host synchronisation anywhere, so bench.py captures the steps into hipGraphs like the scalar
reductions. The slot a step writes holds the global index (int64).
"""
from __future__ import annotations

from typing import Optional

import torch

from .._native import native
from ..ops import KernelConfig, arg_reduce, fill_
from ..ops.reduce import DTYPE_CODES, op_code
from ..parallel import dist as pdist

__all__ = ["LocReduction", "LOC_OPS"]

LOC_OPS = {"maxloc": "max", "minloc": "min"}


def _stream_handle(device: torch.device) -> int:
    return int(torch.cuda.current_stream(device).cuda_stream)


class LocReduction:
    """Global first index (and value) of the maximum / minimum of a sharded array."""

    def __init__(self, cfg, ctx: pdist.DistContext, kernel: Optional[KernelConfig] = None, seed: int = 0x5EED,
                 acc_dtype: Optional[torch.dtype] = None, streams: int = 1, always_collective: bool = False):
        if cfg.op not in LOC_OPS:
            raise ValueError(f"LocReduction needs op maxloc|minloc, got {cfg.op!r}")
        self.cfg = cfg
        self.ctx = ctx
        self.seed = seed
        self.kind = LOC_OPS[cfg.op]
        self.acc = torch.int64  # slots hold global indices
        self.x: Optional[torch.Tensor] = None
        self.offset = self.count = self.n_total = 0
        self.reducer = None
        self.lanes: list = []
        self.plan: Optional[dict] = None
        self.collective = "rccl"
        self.always_collective = bool(always_collective)
        self.channels: list = []

    def setup(self) -> "LocReduction":
        dev = self.ctx.device
        if self.cfg.n_total is None:
            raise ValueError("LocReduction needs a fixed n_total")
        self.n_total = self.cfg.n_total
        self.offset, self.count = pdist.shard(self.n_total, self.ctx.rank, self.ctx.world_size)
        if self.count < 1:
            raise ValueError("every rank needs at least one element")
        self.x = torch.empty(self.count, dtype=self.cfg.dtype, device=dev)
        fill_(self.x, self.cfg.pattern, seed=self.seed, offset=self.offset)
        self.val = torch.empty(1, dtype=self.cfg.dtype, device=dev)
        self.idx = torch.empty(1, dtype=torch.int64, device=dev)
        self._offset_t = torch.tensor([self.offset], dtype=torch.int64, device=dev)
        if dev.type == "cuda":
            self._C = native()
            self._dt = DTYPE_CODES[self.cfg.dtype]
            self._op = op_code(self.kind)
            self._ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            need = self._C.arg_reduce_scratch_bytes(1, self.count, self._dt, self._ncu)
            self._scratch = torch.zeros(max(need, 256), dtype=torch.uint8, device=dev)  # tickets start at 0
            self._pair = torch.empty(2, dtype=torch.int64, device=dev)
            self._pairs = torch.empty(2 * self.ctx.world_size, dtype=torch.int64, device=dev)
            self._device_pick = self.ctx.world_size == 1 or self.ctx.backend == "nccl"
            self.lanes = [(torch.cuda.current_stream(dev), None)]
            torch.cuda.synchronize(dev)
        return self

    @property
    def bytes_total(self) -> int:
        return self.n_total * self.x.element_size()

    def new_slots(self, k: int) -> torch.Tensor:
        return torch.empty(k, dtype=torch.int64, device=self.ctx.device)

    def _local(self) -> None:
        if self.ctx.device.type == "cuda":
            self.plan = self._C.arg_reduce_rows(self.x.data_ptr(), 1, self.count, self._dt, self._op,
                                                self.val.data_ptr(), self.idx.data_ptr(), self._scratch.data_ptr(),
                                                self._ncu, _stream_handle(self.ctx.device))
        else:
            v, i = arg_reduce(self.x, self.kind)
            self.val.copy_(v.reshape(1))
            self.idx.copy_(i.reshape(1))

    def step(self, out: torch.Tensor, async_op: bool = True, corrupt: bool = False):
        """Local arg-reduction, then the cross-rank MAXLOC/MINLOC; writes the global index into
        ``out`` (1 element). ``corrupt`` (fault injection) shifts this rank's local index."""
        self._local()
        if self.ctx.device.type == "cuda" and self._device_pick:
            sh = _stream_handle(self.ctx.device)
            self._C.loc_pack(self.val.data_ptr(), self.idx.data_ptr(), self.offset + (1 if corrupt else 0), self._dt,
                             self._pair.data_ptr(), sh)
            pairs, world = self._pair, 1
            if self.issues_collective:
                torch.distributed.all_gather_into_tensor(self._pairs, self._pair)
                pairs, world = self._pairs, self.ctx.world_size
            self._C.loc_pick(pairs.data_ptr(), world, self._dt, self._op, out.data_ptr(), 0, sh)
            return None
        gi = self.idx + self._offset_t
        if corrupt:
            gi = gi + 1
        if self.issues_collective:
            _, gi = pdist.loc_allreduce(self.val, gi, self.kind)
        out.copy_(gi.reshape(1))
        return None

    @property
    def issues_collective(self) -> bool:
        return self.ctx.world_size > 1 or self.always_collective

    def fork(self) -> None:
        pass

    def join(self) -> None:
        pass

    def check(self):
        return None

    def reference(self) -> int:
        """Independent answer: torch's own argmax/argmin of each shard, combined across ranks."""
        x = self.x
        i = x.argmax() if self.kind == "max" else x.argmin()
        v = x[i].reshape(1)
        gi = (i + self.offset).reshape(1).to(torch.int64)
        if self.ctx.world_size > 1:
            _, gi = pdist.loc_allreduce(v, gi, self.kind)
        return int(gi.item())

    def verify(self, result: torch.Tensor) -> dict:
        got = int(result.reshape(-1)[0].item())
        exp = self.reference()
        return {"ok": got == exp, "got": got, "expected": exp, "tolerance": 0.0}
