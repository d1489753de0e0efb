"""hipGraph replay of independent benchmark steps.

A bench step at N GPUs is a 0.14 ms local reduce plus a 1-element RCCL all-reduce. Issued
eagerly from Python, the all-reduce's stream/event bookkeeping costs ~22 us of GPU-side gaps per
step even on one rank (profiles/r1_bench/host_overhead.jsonl: 0.165 vs 0.141 ms/step at a 1 GB
shard); replaying a captured graph of the same steps brings it back to 0.1417 ms. The reference
had no equivalent (one blocking MPI_Reduce per measurement, mpi/reduce.c:76,90); this is the
"HIP graphs instead of a tracing compiler" part of the MI355X design.

:class:`StepGraph` captures ``chunk`` consecutive steps (each enqueued by ``step_fn(j)``, which may
return a ``torch.distributed`` work handle) into one graph — the all-reduce of step j overlaps
the local reduce of step j+1 inside the graph — plus a remainder graph, so ``run()`` executes
exactly ``n_steps`` steps. With ``serial=True`` every step's work handle is waited on before the
next step is enqueued (the captured graph then has the dependency chain reduce -> all-reduce ->
reduce ..., i.e. every replayed step completes before the next starts: the reference's timing of
one reduction to completion, reduction.cpp:319-374). ``fork`` / ``join`` (optional) are called at
the start / end of every captured chunk (multi-stream steps: fork the side streams off the capture
stream and join them back). All ranks must capture (``capture`` is collective when a process group
is given): capture success is agreed with an all-reduce so either every rank replays graphs or
every rank falls back to eager issue.
"""
from __future__ import annotations

import time
from typing import Callable, Optional

import torch

__all__ = ["StepGraph", "pick_chunk"]


def _nccl_group() -> bool:
    dist = torch.distributed
    return dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"


def pick_chunk(n_steps: int, max_chunk: int = 32) -> int:
    return max(1, min(int(n_steps), int(max_chunk)))


class StepGraph:
    def __init__(self, step_fn: Callable[[int], object], n_steps: int, device: torch.device,
                 chunk: Optional[int] = None, serial: bool = False,
                 fork: Optional[Callable[[], None]] = None, join: Optional[Callable[[], None]] = None):
        self.step_fn = step_fn
        self.serial = bool(serial)
        self.fork = fork
        self.join = join
        self.n_steps = int(n_steps)
        self.device = device
        self.chunk = pick_chunk(self.n_steps) if chunk is None else max(1, min(int(chunk), self.n_steps))
        self.reps, self.rem = divmod(self.n_steps, self.chunk)
        self.graphs: list = []
        self.error: Optional[str] = None

    def _capture_one(self, count: int) -> "torch.cuda.CUDAGraph":
        g = torch.cuda.CUDAGraph()
        # thread_local: HIP calls made by other threads meanwhile (ProcessGroupNCCL's watchdog
        # querying events of earlier eager collectives) must not invalidate this capture.
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            if self.fork is not None:
                self.fork()
            works = []
            for j in range(count):
                w = self.step_fn(j)
                if w is not None:
                    if self.serial:
                        w.wait()
                    else:
                        works.append(w)
            for w in works:
                w.wait()
            if self.join is not None:
                self.join()
        return g

    def capture(self, group_agree: bool = False, settle_s: Optional[float] = None) -> bool:
        """Capture the chunk graph (and the remainder graph). Returns True if graphs will be used.

        ``settle_s`` (default: 0.35 s when a NCCL process group exists, else 0): wait after the
        pre-capture synchronisation so ProcessGroupNCCL's watchdog retires every eager collective
        first. HIP refuses a query of an event recorded on a stream that is capturing at that moment
        (hipErrorCapturedEvent); the watchdog queries the end events of pending eager works every
        ~100 ms and, when one such query fails during our capture — the captured collectives put
        the NCCL stream into the capture — it aborts the whole process (seen in the tuning runs,
        whose 128-step RCCL captures take tens of ms)."""
        ok = True
        prev = torch.cuda.current_stream(self.device)
        if settle_s is None:
            settle_s = 0.35 if _nccl_group() else 0.0
        try:
            torch.cuda.synchronize(self.device)
            if settle_s > 0:
                time.sleep(settle_s)
            self.graphs = [self._capture_one(self.chunk)]
            if self.rem:
                self.graphs.append(self._capture_one(self.rem))
            torch.cuda.synchronize(self.device)
        except Exception as e:  # fall back to eager issue, recorded in the bench JSON
            ok = False
            self.error = f"{type(e).__name__}: {e}"[:300]
            self.graphs = []
            # A capture aborted by an exception leaves torch's capture stream (invalidated) as the
            # current stream — torch.cuda.graph's __exit__ raises before restoring it — so every
            # later launch would fail; restore the caller's stream and clear the thread's HIP error.
            torch.cuda.set_stream(prev)
            from .._native import native
            native().hip_get_last_error()
            torch.cuda.synchronize(self.device)
        if group_agree:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
            if not bool(flag.item()):
                ok = False
                self.error = self.error or "capture failed on another rank"
                self.graphs = []
        return ok

    @property
    def captured(self) -> bool:
        return bool(self.graphs)

    def run(self) -> None:
        """Enqueue exactly n_steps steps (graph replays)."""
        g = self.graphs[0]
        for _ in range(self.reps):
            g.replay()
        if self.rem:
            self.graphs[1].replay()

    def reset(self) -> None:
        """Free the captured graphs. Call before destroying the process group: graphs that captured
        RCCL kernels must not outlive the communicator they reference."""
        for g in self.graphs:
            g.reset()
        self.graphs = []
