"""Direct element-wise collectives over xGMI from Python: :class:`DirectComm`.

The MI355X-native counterpart of mpi/reduce.c's element-wise ``MPI_Reduce`` (reduce.c:76,90) and
of the vendored simpleP2P peer-access pattern (cuda/C/src/simpleP2P/simpleP2P.cu:164,250-330):
every rank maps every peer's registered input / output / signal buffers once (HIP IPC), then a
collective is ONE kernel (csrc/kernels/direct.hip) that pulls this rank's chunk from all peers at
once (reduce-scatter over all 7 xGMI links), meets the peers at device-side per-workgroup barriers
and pulls the other reduced chunks (all-gather) — no RCCL, no host synchronisation, so it can be
captured into a hipGraph.

    comm = DirectComm(device, nbytes)          # collective over the default process group
    comm.allreduce(t, "sum")                   # in place: t <- SUM over ranks of t
    comm.reduce(t, "max", root=0)              # t on root <- MAX over ranks (others: unchanged)
    comm.check()                               # None, or the device-side timeout error

``t`` is staged through the registered buffers (two stream-ordered device copies); for zero-copy
use, write into ``comm.in_view(n, dtype)`` and read ``comm.out_view(n, dtype)``.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .._native import native
from .topology import peer_map

__all__ = ["DirectComm"]


class _CudaArray:
    """Minimal ``__cuda_array_interface__`` holder: lets torch alias a registered buffer."""

    def __init__(self, ptr: int, n: int, dtype: torch.dtype):
        typestr = {torch.float64: "<f8", torch.float32: "<f4", torch.int64: "<i8", torch.int32: "<i4"}[dtype]
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 2}


class DirectComm:
    """Registered peer buffers + the one-kernel direct all-reduce / reduce (collective ctor)."""

    def __init__(self, device: torch.device, nbytes: int, group=None, grid: int = 0, timeout_s: float = 10.0,
                 fault=None):
        """``grid`` 0: one workgroup per CU, divided by the most ranks that share one GPU (every
        rank's workgroups must be co-resident to meet at the device-side barriers; ranks sharing a
        GPU — the one-GPU rehearsals — split its CUs). ``fault`` (:class:`utils.fault.FaultInjector`,
        kind ``mailbox``): that rank fails to register its buffers (the failure-path test)."""
        C = native()
        self.device = torch.device(device)
        self.group = group
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        if dist.is_available() and dist.is_initialized():
            world, rank = dist.get_world_size(group), dist.get_rank(group)
        else:
            world, rank = 1, 0
        if world > 1:
            pm = peer_map(idx, group)  # collective; the same verdict on every rank
            if pm.error:
                raise RuntimeError("direct collective unavailable: " + pm.error)
            if grid <= 0 and pm.ranks_per_gpu > 1:
                grid = max(1, torch.cuda.get_device_properties(idx).multi_processor_count // pm.ranks_per_gpu)
        # Same failure-safe protocol as parallel.xrank.open_channel: every rank reaches every
        # collective, errors are agreed on and raised on all ranks together.
        err, handles = None, b""
        self._d = None
        try:
            if fault is not None and fault.mailbox(rank):
                raise RuntimeError("injected registration failure (--inject-fault mailbox)")
            self._d = C.DirectAllreduce(idx, int(nbytes), int(grid), float(timeout_s))
            handles = self._d.handles()
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        if world > 1:
            allh: list = [None] * world
            dist.all_gather_object(allh, handles, group=group)
        else:
            allh = [handles]
        if err is None:
            if any(not h for h in allh):
                err = "a peer could not register its buffers"
            else:
                try:
                    self._d.connect(rank, world, allh)
                except Exception as e:  # noqa: BLE001
                    err = f"{type(e).__name__}: {e}"
        errs = [err]
        if world > 1:
            errs = [None] * world
            dist.all_gather_object(errs, err, group=group)
        # the ranks that failed themselves first (the others only saw a missing peer)
        own = [f"rank {r}: {m}" for r, m in enumerate(errs) if m and not m.startswith("a peer")]
        bad = own + [f"rank {r}: {m}" for r, m in enumerate(errs) if m and m.startswith("a peer")]
        if bad:
            raise RuntimeError("direct collective unavailable: " + "; ".join(bad)[:500])
        self.rank, self.world = rank, world
        self.nbytes = self._d.bytes
        self.grid = self._d.grid  # workgroups per collective (see ``grid`` above)

    # ------------------------------------------------------------------ buffers
    def in_view(self, n: int, dtype: torch.dtype) -> torch.Tensor:
        """A tensor aliasing the first ``n`` elements of this rank's registered input buffer."""
        self._fits(n, dtype)
        return torch.as_tensor(_CudaArray(self._d.in_ptr, n, dtype), device=self.device)

    def out_view(self, n: int, dtype: torch.dtype) -> torch.Tensor:
        """A tensor aliasing the first ``n`` elements of this rank's registered output buffer."""
        self._fits(n, dtype)
        return torch.as_tensor(_CudaArray(self._d.out_ptr, n, dtype), device=self.device)

    def _fits(self, n: int, dtype: torch.dtype) -> None:
        if n * torch.empty((), dtype=dtype).element_size() > self.nbytes:
            raise ValueError(f"{n} x {dtype} exceeds the {self.nbytes} registered bytes")

    # ------------------------------------------------------------------ collectives
    def launch_allreduce(self, n: int, dtype: torch.dtype, op: str = "sum") -> None:
        """out[:n] <- op over ranks of in[:n] (registered buffers, current stream)."""
        from ..ops.reduce import dtype_code, op_code
        self._fits(n, dtype)
        self._d.allreduce(n, dtype_code(dtype), op_code(op), torch.cuda.current_stream(self.device).cuda_stream)

    def launch_reduce(self, n: int, dtype: torch.dtype, op: str = "sum", root: int = 0) -> None:
        """out[:n] on ``root`` <- op over ranks of in[:n]."""
        from ..ops.reduce import dtype_code, op_code
        self._fits(n, dtype)
        self._d.reduce(n, dtype_code(dtype), op_code(op), root, torch.cuda.current_stream(self.device).cuda_stream)

    def _stage(self, t: torch.Tensor, into_in: bool) -> None:
        C = native()
        s = torch.cuda.current_stream(self.device).cuda_stream
        nb = t.numel() * t.element_size()
        if into_in:
            C.memcpy_d2d(self._d.in_ptr, t.data_ptr(), nb, s)
        else:
            C.memcpy_d2d(t.data_ptr(), self._d.out_ptr, nb, s)

    def allreduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In place: ``t`` <- op over ranks of ``t`` (contiguous, int32/int64/float32/float64)."""
        if not t.is_contiguous() or t.device != self.device:
            raise ValueError("allreduce needs a contiguous tensor on the communicator's device")
        self._stage(t, True)
        self.launch_allreduce(t.numel(), t.dtype, op)
        self._stage(t, False)
        return t

    def reduce(self, t: torch.Tensor, op: str = "sum", root: int = 0) -> torch.Tensor:
        """In place on ``root``: ``t`` <- op over ranks of ``t`` (other ranks' ``t`` unchanged)."""
        if not t.is_contiguous() or t.device != self.device:
            raise ValueError("reduce needs a contiguous tensor on the communicator's device")
        self._stage(t, True)
        self.launch_reduce(t.numel(), t.dtype, op, root)
        if self.rank == root:
            self._stage(t, False)
        return t

    def read_peers(self, nbytes: Optional[int] = None) -> None:
        """Fabric probe (no reduction): one kernel on the current stream reads ``nbytes`` (default:
        all registered bytes) of every peer's input buffer at once over xGMI."""
        nb = self.nbytes if nbytes is None else int(nbytes)
        self._d.read_peers(nb, torch.cuda.current_stream(self.device).cuda_stream)

    def check(self) -> Optional[str]:
        """None if no device-side barrier ever timed out on any rank (collective)."""
        bad = int(self._d.error())
        if self.world > 1:
            t = torch.tensor([bad], dtype=torch.int64)
            if dist.get_backend(self.group) == "nccl":
                t = t.to(self.device)
            dist.all_reduce(t, group=self.group)
            bad = int(t.item())
        return None if bad == 0 else f"direct collective: {bad} rank(s) timed out at a device-side barrier"

    @property
    def epoch(self) -> int:
        return int(self._d.epoch())

    def close(self) -> None:
        """Collective teardown: unmap the peers' buffers, free this rank's, then wait for every rank.
        A registration that follows (here or on a peer) may get the same addresses back, and its
        IPC export failed while a peer still mapped the old buffer at that address (seen in the
        bench's back-to-back registrations); after the barrier nobody does."""
        if self._d is not None:
            torch.cuda.synchronize(self.device)
            self._d = None  # native destructor: close peer mappings, free own buffers
        if self.world > 1:
            if dist.get_backend(self.group) == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)
