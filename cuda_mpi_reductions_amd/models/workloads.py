"""Benchmark workloads — the "models" of a reduction framework.

The reference has no neural model; its runnable artefacts are two benchmarks:
* ``reduction --method=... --type=...`` — one array reduced to one scalar on one GPU
  (cuda/C/src/reduction/reduction.cpp:84-204, 661-783);
* ``reduce`` — element-wise vector ``MPI_Reduce`` of an N/P shard per rank to root 0
  (mpi/reduce.c:9-108).

Here both semantics are workloads with a common ``setup / step / verify`` life-cycle, and the
five BASELINE.json configs are registered in :data:`CONFIGS`. A *step* of
:class:`ScalarReduction` is: local HIP reduction of this rank's shard into a 1-element slot,
then an RCCL all-reduce of that slot over xGMI (SURVEY.md §5.8 "mode scalar").
"""
from __future__ import annotations

import contextlib
import math
from dataclasses import dataclass
from typing import Optional

import torch

from ..ops import KernelConfig, Reducer, default_acc_dtype, fill_, sum_tolerance
from ..parallel import dist as pdist

__all__ = ["WorkloadConfig", "CONFIGS", "NORTH_STAR", "COLLECTIVES", "VECTOR_IMPLS", "ScalarReduction", "VectorReduction",
           "element_size"]


@dataclass(frozen=True)
class WorkloadConfig:
    name: str
    dtype: torch.dtype
    op: str
    n_total: Optional[int]          # None: size each GPU's shard to fill its HBM
    mode: str = "scalar"            # "scalar" (array -> one value) | "vector" (reduce.c)
    collective: str = "allreduce"   # "allreduce" | "reduce"
    pattern: str = "uniform"
    device: str = "cuda"
    baseline: Optional[float] = None
    baseline_unit: str = "GB/s"
    baseline_source: str = ""
    description: str = ""
    hbm_fraction: float = 0.96      # share of free HBM used when n_total is None


def element_size(dt: torch.dtype) -> int:
    return torch.empty((), dtype=dt).element_size()


CONFIGS: dict[str, WorkloadConfig] = {
    "mpi_1m_int32_sum_cpu2": WorkloadConfig(
        name="mpi_1m_int32_sum_cpu2", dtype=torch.int32, op="sum", n_total=1 << 20,
        mode="vector", collective="reduce", pattern="fullrange", device="cpu",
        description="1M int32 sum via MPI_Reduce on 2 CPU ranks (reduce.c plumbing, no GPU)",
    ),
    "xgmi_2g_double_sum_reduce": WorkloadConfig(
        name="xgmi_2g_double_sum_reduce", dtype=torch.float64, op="sum", n_total=256 * 1024 * 1024,
        mode="vector", collective="reduce", baseline=60.97540, baseline_unit="GiB/s",
        baseline_source="mpi/results/DOUBLE_SUM.txt:2 (MPI_Reduce DOUBLE SUM, BG/L 1024 ranks)",
        description="reduce.c on GPUs: element-wise DOUBLE SUM of NUM_DOUBLES (2 GiB total) to root 0, "
                    "N/P per rank (mpi/reduce.c:90, mpi/constants.h:2)",
    ),
    "xgmi_2g_int_sum_reduce": WorkloadConfig(
        name="xgmi_2g_int_sum_reduce", dtype=torch.int32, op="sum", n_total=512 * 1024 * 1024,
        mode="vector", collective="reduce", pattern="fullrange", baseline=146.81800, baseline_unit="GiB/s",
        baseline_source="mpi/results/INT_SUM.txt:2 (MPI_Reduce INT SUM, BG/L 1024 ranks)",
        description="reduce.c on GPUs: element-wise INT SUM of NUM_INTS (2 GiB total) to root 0, N/P per "
                    "rank (mpi/reduce.c:76, mpi/constants.h:1)",
    ),
    "gpu_256m_double_sum": WorkloadConfig(
        name="gpu_256m_double_sum", dtype=torch.float64, op="sum", n_total=256 * 1024 * 1024,
        baseline=92.7729, baseline_source="mpi/CUdata.txt:2 (CUDA DOUBLE SUM)",
        description="256M double sum on one MI355X (single-GPU HIP tree-reduction kernel)",
    ),
    "gpu_256m_int64_min": WorkloadConfig(
        name="gpu_256m_int64_min", dtype=torch.int64, op="min", n_total=256 * 1024 * 1024,
        baseline=92.6014, baseline_source="mpi/CUdata.txt:3 (CUDA DOUBLE MIN; reference has no int64)",
        description="256M int64 min-reduce on one MI355X (non-sum op path)",
    ),
    "xgmi_1b_double_sum": WorkloadConfig(
        name="xgmi_1b_double_sum", dtype=torch.float64, op="sum", n_total=1_000_000_000,
        baseline=92.7729, baseline_source="mpi/CUdata.txt:2 (CUDA DOUBLE SUM, best reference GB/s)",
        description="1B double sum across N MI355X: local HIP reduce + cross-rank combine over xGMI "
                    "(fused in-kernel mailbox exchange, or a 1-element RCCL all-reduce)",
    ),
    "xgmi_1b_double_norm2": WorkloadConfig(
        name="xgmi_1b_double_norm2", dtype=torch.float64, op="sumsq", n_total=1_000_000_000,
        description="sum of squares (squared L2 norm) of 1e9 doubles across N GPUs, square fused into the "
                    "load (MI355X addition; not a reference config)",
    ),
    "xgmi_1b_double_maxloc": WorkloadConfig(
        name="xgmi_1b_double_maxloc", dtype=torch.float64, op="maxloc", n_total=1_000_000_000,
        description="MPI_MAXLOC of 1e9 doubles across N GPUs: local arg-reduction + all-gather of (value, "
                    "index) pairs over RCCL (MI355X addition; not a reference config)",
    ),
    "gpu_4g_bf16_sum": WorkloadConfig(
        name="gpu_4g_bf16_sum", dtype=torch.bfloat16, op="sum", n_total=4_000_000_000,
        description="4e9 bfloat16 (8 GB) sum, fp32 accumulation (MI355X addition; not a reference config)",
    ),
    "hbm_fill_fp32_sum": WorkloadConfig(
        name="hbm_fill_fp32_sum", dtype=torch.float32, op="sum", n_total=None,
        description="fp32 sum with each GPU's shard sized to fill its 288 GB HBM (HBM saturation)",
    ),
}

NORTH_STAR = "xgmi_1b_double_sum"


_nullcontext = contextlib.nullcontext
_CPU_CHANNELS = [0]  # CPU twin channels opened by this process (every rank opens them in the same order)


def _current_stream_handle(device: torch.device) -> int:
    try:
        return torch._C._cuda_getCurrentRawStream(device.index)
    except AttributeError:  # older torch
        return int(torch.cuda.current_stream(device).cuda_stream)


COLLECTIVES = ("rccl", "fused")


class ScalarReduction:
    """Global reduction of a sharded array to one value on every rank.

    ``collective`` picks how the ranks' partials are combined:

    * ``"rccl"`` — the local single-pass kernel writes this rank's partial, then a 1-element
      ``torch.distributed`` all-reduce (RCCL over xGMI) combines them (a second kernel, on RCCL's
      stream);
    * ``"fused"`` — the local kernel's last workgroup exchanges the partials through IPC-mapped
      mailboxes and writes the global value itself (:mod:`parallel.xrank`): one kernel per step.

    ``always_collective``: issue the cross-rank combine even on a single rank (the bench and the
    smoke test run the exact N-GPU step on one GPU this way).
    ``streams`` > 1 alternates independent steps over that many HIP streams ("lanes"), each with
    its own workspace (and channel), so one step's tail overlaps the next step's body.
    """

    def __init__(self, cfg: WorkloadConfig, ctx: pdist.DistContext,
                 kernel: Optional[KernelConfig] = None, seed: int = 0x5EED,
                 acc_dtype: Optional[torch.dtype] = None, streams: int = 1,
                 collective: str = "rccl", always_collective: bool = False,
                 xrank_timeout_s: float = 10.0, fault=None):
        if cfg.mode != "scalar":
            raise ValueError("ScalarReduction needs a scalar-mode config")
        if collective not in COLLECTIVES:
            raise ValueError(f"collective must be one of {COLLECTIVES}, got {collective!r}")
        self.cfg = cfg
        self.ctx = ctx
        self.kernel = kernel or KernelConfig()
        self.seed = seed
        self.acc = acc_dtype or default_acc_dtype(cfg.dtype, cfg.op)
        self.collective = collective
        self.always_collective = bool(always_collective)
        self.xrank_timeout_s = xrank_timeout_s
        self.fault = fault  # FaultInjector: a "mailbox" fault fails this rank's channel creation
        self.x: Optional[torch.Tensor] = None
        self.offset = 0
        self.count = 0
        self.n_total = 0
        self.reducer: Optional[Reducer] = None
        self.n_streams = max(1, int(streams))
        # lanes[k] = (stream, reducer, bound launch, xrank channel or None); lane 0 runs on the
        # caller's current stream when there is a single lane.
        self.lanes: list = []
        self.channels: list = []
        self._next = 0
        self._fork = None
        self.bound = None  # lane 0's prepared launch, set by setup()
        self._local_bound = None  # lane 0's plan without a channel (local_step), made on first use
        self._cpu_xrank = None  # CPU ranks: the fused finish's twin channel (_open_cpu_channel)

    # ------------------------------------------------------------------ setup
    def _size_for_hbm(self) -> int:
        free_b, _ = torch.cuda.mem_get_info(self.ctx.device)
        es = element_size(self.cfg.dtype)
        n = int(free_b * self.cfg.hbm_fraction) // es
        return n - n % 64

    def setup(self) -> "ScalarReduction":
        dev = self.ctx.device
        if self.cfg.n_total is None:
            if dev.type != "cuda":
                raise RuntimeError("HBM-fill config needs GPUs")
            per_rank = self._size_for_hbm()
            t = torch.tensor([per_rank], dtype=torch.int64, device=dev)
            if self.ctx.world_size > 1:
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
            per_rank = int(t.item())
            self.n_total = per_rank * self.ctx.world_size
            self.offset, self.count = self.ctx.rank * per_rank, per_rank
        else:
            self.n_total = self.cfg.n_total
            self.offset, self.count = pdist.shard(self.n_total, self.ctx.rank, self.ctx.world_size)
        self.x = torch.empty(self.count, dtype=self.cfg.dtype, device=dev)
        fill_(self.x, self.cfg.pattern, seed=self.seed, offset=self.offset)
        if dev.type == "cuda":
            if self.collective == "fused":
                from ..parallel.xrank import open_channel
            self._bound_out = self.new_slots(1)  # default target; steps pass their own slot
            for k in range(self.n_streams):
                stream = torch.cuda.current_stream(dev) if self.n_streams == 1 else torch.cuda.Stream(dev)
                reducer = Reducer(dev, config=self.kernel)
                ch = open_channel(dev, timeout_s=self.xrank_timeout_s, fault=self.fault) \
                    if self.collective == "fused" else None
                bound = reducer.bind(self.x, self.cfg.op, self.acc, out=self._bound_out, xrank=ch)
                self.lanes.append((stream, reducer, bound, ch))
                if ch is not None:
                    self.channels.append(ch)
            self.reducer, self.bound = self.lanes[0][1], self.lanes[0][2]
            torch.cuda.synchronize(dev)
        elif self.collective == "fused":
            self._open_cpu_channel()
        return self

    # ------------------------------------------------------------------ the fused finish's CPU twin
    def _open_cpu_channel(self) -> None:
        """CPU ranks (bench.py --rehearse-stages, tests): a twin of the fused cross-rank finish with
        the same protocol and failure semantics as the in-kernel one (xrank.hpp): every step's
        partial is pushed into a per-launch mailbox (a key of the job's rendezvous store, tagged with
        the channel and the launch epoch), the peers' are waited for at most ``xrank_timeout_s``
        (then the result is poisoned and the sticky error set; later launches look once) and folded
        in rank order. Opening is collective and agreed (a rank failing to create its mailbox — the
        ``mailbox`` fault — fails every rank's open, as ``parallel.xrank.open_channel`` does)."""
        _CPU_CHANNELS[0] += 1
        ok = self.fault is None or not self.fault.mailbox(self.ctx.rank)
        rows = pdist.agree(self.ctx, "xrank open", {"ok": ok}, timeout_s=max(30.0, self.xrank_timeout_s))
        bad = [r for r, row in enumerate(rows) if not row["ok"]]
        if bad:
            self._cpu_xrank = None
            raise RuntimeError(f"fused finish (CPU twin): rank(s) {bad} could not create a mailbox")
        self._cpu_xrank = {"id": _CPU_CHANNELS[0], "epoch": 0, "err": 0}

    def _poisoned(self) -> float:
        if self.acc.is_floating_point:
            return float("nan")
        info = torch.iinfo(self.acc)
        return {"min": info.max, "max": info.min}.get(self.cfg.op, 0)

    def _cpu_exchange(self, out: torch.Tensor) -> None:
        ch = self._cpu_xrank
        ch["epoch"] += 1
        if self.ctx.world_size == 1:
            return
        import datetime
        import json
        store = pdist._store()
        base = f"mireduce/xrank/{ch['id']}/{ch['epoch']}/"
        store.set(base + str(self.ctx.rank), json.dumps(out.reshape(-1)[0].item()))
        keys = [base + str(r) for r in range(self.ctx.world_size)]
        limit = 0.001 if ch["err"] else self.xrank_timeout_s  # a sticky error: a peer is gone, look once
        try:
            store.wait(keys, datetime.timedelta(seconds=limit))
        except Exception:  # noqa: BLE001 - a peer's partial missed the timeout
            ch["err"] |= 1
            out.fill_(self._poisoned())
            return
        vals = [json.loads(store.get(k)) for k in keys]
        op = self.cfg.op
        acc = vals[0]
        for v in vals[1:]:  # rank order: deterministic, like the kernel's lane-ordered fold
            acc = min(acc, v) if op == "min" else max(acc, v) if op in ("max", "amax") else acc + v
        out.fill_(acc)

    def use_collective(self, collective: str, streams: Optional[int] = None) -> None:
        """Re-bind for another cross-rank combine (e.g. fall back from ``fused`` to ``rccl``) and/or
        another number of stream lanes, keeping the data. Collective when the result is ``fused``
        (every rank must call it with the same arguments)."""
        if collective not in COLLECTIVES:
            raise ValueError(f"collective must be one of {COLLECTIVES}")
        if self.ctx.device.type != "cuda":
            self._cpu_xrank = None
            self.collective = collective
            if collective == "fused":
                self._open_cpu_channel()
            return
        dev = self.ctx.device
        torch.cuda.synchronize(dev)
        n = self.n_streams if streams is None else max(1, int(streams))
        from ..parallel.xrank import close_channels, open_channel
        old = [(st, red) for st, red, _, _ in self.lanes]  # keep streams and workspaces
        # Drop every reference to the old bound reductions and channels, then tear the channels
        # down collectively (a new mailbox may reuse an old one's address; see close_channels).
        self.lanes, self.bound, self._local_bound = [], None, None
        close_channels(self.channels, dev)
        lanes, channels = [], []
        for k in range(n):
            if n == 1:
                stream = torch.cuda.current_stream(dev)
            else:
                stream = old[k][0] if len(old) > 1 and k < len(old) else torch.cuda.Stream(dev)
            reducer = old[k][1] if k < len(old) and old[k][1].config == self.kernel else Reducer(dev, config=self.kernel)
            ch = open_channel(dev, timeout_s=self.xrank_timeout_s, fault=self.fault) if collective == "fused" else None
            bound = reducer.bind(self.x, self.cfg.op, self.acc, out=self._bound_out, xrank=ch)
            lanes.append((stream, reducer, bound, ch))
            if ch is not None:
                channels.append(ch)
        self.lanes, self.channels = lanes, channels
        self.n_streams = n
        self._next = 0
        self.reducer, self.bound = lanes[0][1], lanes[0][2]
        self.collective = collective
        torch.cuda.synchronize(dev)

    def use_kernel(self, kernel: KernelConfig, streams: Optional[int] = None) -> None:
        """Re-bind every lane with another streaming-kernel plan (fresh reducers; same data and
        combine). LOCAL, also with the fused finish: each lane keeps its channel, whose mailboxes,
        epoch counter and error word belong to the exchange, not to the plan (every rank still makes
        one fused launch per step, so the epochs stay in step), so ranks may re-plan each on their
        own and no rank can be left waiting in a collective (bench.py's per-rank plan tuning).
        Changing the number of lanes goes through :meth:`use_collective` (collective when fused).
        As with :meth:`use_collective`, graphs captured from the old lanes must not be replayed after
        it (their workspaces are released)."""
        self.kernel = kernel
        n = self.n_streams if streams is None else max(1, int(streams))
        if self.ctx.device.type != "cuda":
            return  # CPU ranks reduce on the host: no plan to bind
        if n != len(self.lanes) or not self.lanes:
            self.use_collective(self.collective, streams=streams)
            return
        dev = self.ctx.device
        torch.cuda.synchronize(dev)
        lanes = []
        for stream, _red, _bound, ch in self.lanes:
            reducer = Reducer(dev, config=kernel)
            lanes.append((stream, reducer, reducer.bind(self.x, self.cfg.op, self.acc, out=self._bound_out, xrank=ch), ch))
        self.lanes, self._local_bound, self._next = lanes, None, 0
        self.reducer, self.bound = lanes[0][1], lanes[0][2]
        torch.cuda.synchronize(dev)

    @property
    def bytes_total(self) -> int:
        return self.n_total * element_size(self.cfg.dtype)

    @property
    def issues_collective(self) -> bool:
        """Whether a step issues an RCCL / gloo collective (the fused finish is in-kernel)."""
        return self.collective == "rccl" and (self.ctx.world_size > 1 or self.always_collective)

    # ------------------------------------------------------------------ step
    def new_slots(self, k: int) -> torch.Tensor:
        return torch.empty(k, dtype=self.acc, device=self.ctx.device)

    def local(self, out: torch.Tensor) -> torch.Tensor:
        """This rank's partial only (no cross-rank combine; never through a fused channel)."""
        if self.ctx.device.type == "cuda":  # an unbound launch on lane 0's workspace: no channel
            return self.reducer(self.x, self.cfg.op, self.acc, out=out)
        from ..ops import reduce as host_reduce
        return host_reduce(self.x, self.cfg.op, self.acc, out=out)

    def local_step(self, out: torch.Tensor, async_op: bool = True, corrupt: bool = False):
        """The step with the combine removed: the SAME kernel plan as :meth:`step` on lane 0's
        workspace and stream, but bound without a channel (one prepared launch, capturable), so
        ``step time - local_step time`` is what the cross-rank exchange costs (bench.py's
        decomposition). Returns None (nothing to wait on)."""
        if self.ctx.device.type != "cuda":
            self.local(out)
        else:
            if self._local_bound is None:
                keep = dict(self.reducer.last_plan)
                self._local_bound = self.reducer.bind(self.x, self.cfg.op, self.acc, out=self._bound_out)
                self.reducer.last_plan = keep  # the record describes the step's launch
            self._local_bound.launch(_current_stream_handle(self.ctx.device), out.data_ptr())
        if corrupt:
            out.sub_(1) if self.cfg.op == "min" else out.add_(1)
        return None

    def local_launcher(self, kernel: KernelConfig):
        """(launch, error) for this rank's local reduction with another streaming-kernel plan —
        ``launch(out)`` enqueues it on the current stream (one prepared launch on a workspace of
        its own, no channel: capturable), ``error()`` reads that workspace's sticky fan-in error word.
        Purely local (no collective, the bound combine untouched): bench.py's per-rank plan tuning
        measures candidates with it on every rank independently."""
        if self.ctx.device.type != "cuda":
            return (lambda out: self.local(out)), (lambda: 0)
        red = Reducer(self.ctx.device, config=kernel)
        bound = red.bind(self.x, self.cfg.op, self.acc, out=self._bound_out)
        dev = self.ctx.device

        def launch(out: torch.Tensor) -> None:
            bound.launch(_current_stream_handle(dev), out.data_ptr())
        launch.plan = red.last_plan  # (the record of a candidate)
        return launch, (lambda: int(red.ws.error()))

    def fork(self) -> None:
        """Multi-lane steps: make every lane's stream follow the caller's current stream (call
        before a batch of steps; inside a graph capture this is the fork of the captured DAG)."""
        if len(self.lanes) > 1:
            cur = torch.cuda.current_stream(self.ctx.device)
            for stream, *_ in self.lanes:
                stream.wait_stream(cur)

    def join(self) -> None:
        """Multi-lane steps: make the caller's current stream wait for every lane."""
        if len(self.lanes) > 1:
            cur = torch.cuda.current_stream(self.ctx.device)
            for stream, *_ in self.lanes:
                cur.wait_stream(stream)

    def step(self, out: torch.Tensor, async_op: bool = True, corrupt: bool = False):
        """Local reduce into ``out`` (1 element) then the cross-rank combine. Returns the RCCL
        collective's work handle, or ``None`` (fused finish, or a single rank without
        ``always_collective``). ``corrupt`` (fault injection) perturbs the local result before
        the collective; verification must catch it (rccl only)."""
        if self.ctx.device.type != "cuda":
            self.local(out)
            if corrupt:
                out.sub_(1) if self.cfg.op == "min" else out.add_(1)
            if self.collective == "fused" and self._cpu_xrank is not None:
                self._cpu_exchange(out)
                return None
            return pdist.scalar_allreduce(out, self.cfg.op, async_op=async_op) if self.issues_collective else None
        stream, _, bound, _ = self.lanes[self._next % len(self.lanes)]
        self._next += 1
        ctx = torch.cuda.stream(stream) if len(self.lanes) > 1 else _nullcontext()
        with ctx:
            bound.launch(_current_stream_handle(self.ctx.device), out.data_ptr())
            if corrupt:
                out.sub_(1) if self.cfg.op == "min" else out.add_(1)
            if self.issues_collective:
                return pdist.scalar_allreduce(out, self.cfg.op, async_op=async_op)
        return None

    def error_counts(self) -> list:
        """This rank's device-side error words as counts, read locally (no collective):
        [workspaces whose polled fan-in reached its bound, workspaces that saw a late XCD anchor,
        channels that timed out waiting for a peer, channels that received a poisoned partial]."""
        if self.ctx.device.type != "cuda":
            late = 1 if self._cpu_xrank is not None and self._cpu_xrank["err"] & 1 else 0
            return [0, 0, late, 0]
        torch.cuda.synchronize(self.ctx.device)
        fan_words = [int(red.ws.error()) for _, red, _, _ in self.lanes]
        words = [int(ch.error()) for ch in self.channels]
        return [sum(int(w != 0) for w in fan_words), sum(int(w & 2 != 0) for w in fan_words),
                sum(int(w & 1 != 0) for w in words), sum(int(w & 2 != 0) for w in words)]

    def reset_fanin(self) -> None:
        """Clear the sticky fan-in errors of every lane's workspace (after they were reported)."""
        if self.ctx.device.type != "cuda":
            return
        dev = self.ctx.device
        for _, red, _, _ in self.lanes:
            red.ws.reset(_current_stream_handle(dev))
        torch.cuda.synchronize(dev)

    @staticmethod
    def describe_errors(counts) -> Optional[str]:
        """The message for (summed) :meth:`error_counts`; None when all are zero."""
        fan, anchor, late, pois = (int(v) for v in counts)
        msgs = []
        if fan:
            msgs.append(f"polled fan-in: {fan} workspace(s) reached the wait bound (results poisoned; reset)")
        if anchor:
            msgs.append(f"XCD-weighted split: {anchor} workspace(s) saw a late XCD anchor (tiles not the split's; "
                        "results poisoned)")
        if late:
            msgs.append(f"fused cross-rank finish: {late} channel(s) timed out waiting for a peer")
        if pois:
            msgs.append(f"fused cross-rank finish: {pois} channel(s) received a peer's poisoned partial "
                        "(its fan-in failed; results poisoned on every rank)")
        return "; ".join(msgs) or None

    def check(self) -> Optional[str]:
        """None, or what went wrong in the launches so far, agreed over ranks (collective when a
        process group spans several ranks; call after the launches):

        * the polled fan-in's sticky error (a launch's finisher reached its wait bound: that launch
          and every later one on the workspace wrote a poisoned result; the workspaces are reset);
        * the fused finish's error words (a peer's partial never arrived, or arrived poisoned
          because that peer's fan-in failed — then every rank's result is poisoned too)."""
        counts = self.error_counts()
        if self.ctx.world_size > 1:
            dev = self.ctx.device
            t = torch.tensor(counts, dtype=torch.int64, device=dev if self.ctx.backend == "nccl" else "cpu")
            torch.distributed.all_reduce(t)
            counts = [int(v) for v in t.tolist()]
        if counts[0]:
            self.reset_fanin()
        return self.describe_errors(counts)

    # ------------------------------------------------------------------ verify
    def reference(self, chunk: int = 1 << 24):
        """Independent global result: torch's own reduction of each shard (in chunks, so HBM-filling
        arrays need no full-size temporaries), combined across ranks in fp64 / int64 (parity: the
        CPU check of reduction.cpp:748-780). The chunks stay small (16M elements: <= 128 MB fp64
        temporaries): releasing GB-sized temporaries to the driver (``empty_cache``, which every
        graph capture calls) slowed the streaming kernel after it by ~6 % (tools/settle_probe.py,
        profiles/r3_selfcheck/)."""
        x = self.x
        dev = x.device
        if self.cfg.op == "sum":
            acc_dt = torch.float64 if x.dtype.is_floating_point else torch.int64
            loc = torch.zeros(1, dtype=acc_dt, device=dev)
            absl = torch.zeros(1, dtype=torch.float64, device=dev)
            for i in range(0, x.numel(), chunk):
                c = x[i:i + chunk]
                loc += c.sum(dtype=acc_dt)
                absl += c.abs().sum(dtype=torch.float64) if c.dtype.is_floating_point else \
                    c.abs().to(torch.float64).sum()
        elif self.cfg.op == "sumsq":  # Σ x² in fp64; every term is non-negative, so Σ|.| is the sum
            loc = torch.zeros(1, dtype=torch.float64, device=dev)
            for i in range(0, x.numel(), chunk):
                c = x[i:i + chunk].double()
                loc += (c * c).sum()
            absl = loc.clone()
        elif self.cfg.op == "amax":
            parts = [x[i:i + chunk].abs().max().reshape(1) for i in range(0, x.numel(), chunk)]
            loc = torch.cat(parts).max().reshape(1).to(self.acc)
            absl = torch.zeros(1, dtype=torch.float64, device=dev)
        else:
            parts = [(x[i:i + chunk].min() if self.cfg.op == "min" else x[i:i + chunk].max()).reshape(1)
                     for i in range(0, x.numel(), chunk)]
            st = torch.cat(parts)
            loc = (st.min() if self.cfg.op == "min" else st.max()).reshape(1)
            absl = torch.zeros(1, dtype=torch.float64, device=dev)
        if self.ctx.world_size > 1:
            torch.distributed.all_reduce(loc, op=pdist.reduce_op(self.cfg.op))
            torch.distributed.all_reduce(absl)
        return loc.item(), absl.item()

    def verify(self, result: torch.Tensor) -> dict:
        got = result.reshape(-1)[0].item()
        exp, abs_sum = self.reference()
        if self.cfg.op in ("sum", "sumsq") and self.acc.is_floating_point:
            tol = sum_tolerance(self.cfg.dtype, self.acc, self.n_total, abs_sum)
            ok = math.isfinite(got) and abs(got - exp) <= tol
        else:
            tol = 0.0
            ok = got == exp
        return {"ok": bool(ok), "got": got, "expected": exp, "tolerance": tol}


VECTOR_IMPLS = ("rccl", "direct")


class VectorReduction:
    """reduce.c semantics: each rank holds N/P elements; element-wise reduce to root 0 (or all).

    ``impl``: ``"rccl"`` — ``torch.distributed`` reduce / all_reduce (RCCL on GPUs, gloo on CPUs);
    ``"direct"`` — the one-kernel peer-read collective over xGMI (:class:`parallel.DirectComm`,
    GPUs only): x is staged into the registered input buffer by ``restore()`` (outside the clock,
    like reduce.c's bzero) and the result read back from the registered output by ``verify()``.
    """

    def __init__(self, cfg: WorkloadConfig, ctx: pdist.DistContext, seed: int = 0x5EED, impl: str = "rccl",
                 direct_grid: int = 0, direct_timeout_s: float = 10.0):
        if impl not in VECTOR_IMPLS:
            raise ValueError(f"impl must be one of {VECTOR_IMPLS}")
        self.cfg = cfg
        self.ctx = ctx
        self.seed = seed
        self.impl = impl
        self.direct_grid = direct_grid
        self.direct_timeout_s = direct_timeout_s
        self.count = cfg.n_total // ctx.world_size if cfg.n_total else 0
        self.x: Optional[torch.Tensor] = None
        self.y: Optional[torch.Tensor] = None
        self.comm = None

    def setup(self, mt19937: bool = False) -> "VectorReduction":
        dev = self.ctx.device
        self.x = torch.empty(self.count, dtype=self.cfg.dtype, device="cpu" if mt19937 else dev)
        if mt19937:
            from ..ops import mt19937_fill_
            mt19937_fill_(self.x, self.ctx.rank)
            self.x = self.x.to(dev)
        else:
            # per-rank distinct streams, like reduce.c's rank-seeded generator
            fill_(self.x, self.cfg.pattern, seed=self.seed + self.ctx.rank, offset=0)
        self.y = torch.empty_like(self.x)
        if self.impl == "direct":
            if dev.type != "cuda":
                raise RuntimeError("the direct collective needs GPUs")
            from ..parallel.direct import DirectComm
            self.comm = DirectComm(dev, max(16, self.x.numel() * self.x.element_size()),
                                   grid=self.direct_grid, timeout_s=self.direct_timeout_s)
        return self

    @property
    def bytes_total(self) -> int:
        # reduce.c counts the full NUM_INTS*sizeof(int) regardless of P (mpi/reduce.c:79,93);
        # we count the bytes actually reduced (count * P), which equals it when P divides N.
        return self.count * self.ctx.world_size * element_size(self.cfg.dtype)

    def restore(self) -> None:
        """Reset the in-place collective buffer (reduce.c's bzero of the receive buffer)."""
        if self.comm is not None:
            from .._native import native
            native().memcpy_d2d(self.comm._d.in_ptr, self.x.data_ptr(), self.x.numel() * self.x.element_size(),
                                torch.cuda.current_stream(self.ctx.device).cuda_stream)
        else:
            self.y.copy_(self.x)

    def collective(self, async_op: bool = False):
        if self.comm is not None:
            if self.cfg.collective == "reduce":
                self.comm.launch_reduce(self.count, self.cfg.dtype, self.cfg.op, root=0)
            else:
                self.comm.launch_allreduce(self.count, self.cfg.dtype, self.cfg.op)
            return None
        if self.cfg.collective == "reduce":
            return pdist.vector_reduce(self.y, self.cfg.op, root=0, async_op=async_op)
        return pdist.vector_allreduce(self.y, self.cfg.op, async_op=async_op)

    def corrupt(self) -> None:
        """Fault injection: this rank's staged contribution at element 0 becomes wrong (the clean
        ``x`` still defines the expected result, so verification must fail)."""
        if self.comm is not None:
            from .._native import native
            bad = self.x[:1] + 1
            native().memcpy_d2d(self.comm._d.in_ptr, bad.data_ptr(), bad.element_size(),
                                torch.cuda.current_stream(self.ctx.device).cuda_stream)
        else:
            self.y.view(-1)[0] += 1

    def result(self) -> torch.Tensor:
        """This rank's result buffer (meaningful on the holders: root for reduce, all for allreduce)."""
        if self.comm is not None:
            from .._native import native
            native().memcpy_d2d(self.y.data_ptr(), self.comm._d.out_ptr, self.y.numel() * self.y.element_size(),
                                torch.cuda.current_stream(self.ctx.device).cuda_stream)
        return self.y

    def step(self, async_op: bool = False):
        self.restore()
        return self.collective(async_op=async_op)

    def close(self) -> None:
        """Collective: release the direct collective's registered buffers (``DirectComm.close``) so
        a following registration on any rank cannot race a peer still mapping them."""
        if self.comm is not None:
            self.comm.close()
            self.comm = None

    VERIFY_CHUNK = 1 << 25  # elements per rank per verification all-gather

    def _check_chunk(self, st: torch.Tensor, y: torch.Tensor, world: int) -> bool:
        if self.cfg.op == "sum":
            if st.dtype.is_floating_point:
                exp = st.double().sum(0)
                tol = 1e-12 * world * (exp.abs() + 1.0)
                return bool(((y.double() - exp).abs() <= tol).all())
            bits = 8 * st.element_size()
            exp = st.long().sum(0) if bits == 32 else st.sum(0)
            if bits == 32:
                exp = ((exp + 2 ** 31) % 2 ** 32 - 2 ** 31).to(st.dtype)
            return bool(torch.equal(exp, y))
        exp = st.min(0).values if self.cfg.op == "min" else st.max(0).values
        return bool(torch.equal(exp, y))

    def verify(self) -> dict:
        """Gather every rank's input (in chunks) and combine on the result holders; integer SUM wraps
        like MPI_INT / ncclInt32 (two's complement)."""
        self.result()
        world = self.ctx.world_size
        holder = self.cfg.collective == "allreduce" or self.ctx.rank == 0
        ok = True
        # In chunks (bounded memory on the holder: world x chunk, widened). gloo gathers host
        # copies: its own GPU-tensor path ran out of host allocations (std::bad_alloc) in the
        # 2-rank reduce.c INT rehearsal on one GPU and left the other rank in a mismatched collective.
        host = world > 1 and self.ctx.backend == "gloo" and self.x.is_cuda
        step = self.VERIFY_CHUNK
        for a in range(0, self.x.numel(), step):
            xs, ys = self.x[a:a + step], self.y[a:a + step]
            if host:
                xs, ys = xs.cpu(), ys.cpu()
            gathered = [torch.empty_like(xs) for _ in range(world)]
            if world > 1:
                torch.distributed.all_gather(gathered, xs.contiguous())
            else:
                gathered[0].copy_(xs)
            if holder and ok:
                ok = self._check_chunk(torch.stack(gathered), ys, world)
        dev_err = self.comm.check() if self.comm is not None else None  # collective
        if dev_err is not None:
            ok = False
        t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                         device=self.ctx.device if self.ctx.backend == "nccl" else "cpu")
        if world > 1:
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
        out = {"ok": bool(t.item())}
        if dev_err is not None:
            out["device_error"] = dev_err
        return out
