#!/usr/bin/env python3
"""Headline benchmark: reduction bandwidth (GB/s, whole node), 1B-double SUM on N MI355X.

Driver contract: ``python bench.py --gpus N --steps K --warmup W`` (N>1 under
``torch.distributed.run``, one rank per GPU, RCCL over xGMI). One *step* is one complete global
reduction of the 1e9-element float64 array (BASELINE.json config 4): every rank reduces its
contiguous 1e9/N shard with the native single-pass HIP kernel (csrc/kernels/reduce_kernels.hpp) into a
1-element slot, and the N partials are combined across ranks (``--collective`` below). The array is
synthetic (on-device counter-based U[0,1) fill, untimed) and fixed in size as N grows -> strong
scaling.

Timing: W untimed warm-up steps; then barrier + synchronize, K timed steps, synchronize; the
MAX elapsed time over ranks defines the measurement. Value = total bytes reduced per step x K /
elapsed / 1e9 (GB = 1e9 B, the CUDA sample's unit, reduction.cpp:744-745).

Cross-rank combine (``--collective``): ``fused`` = the local kernel's last workgroup exchanges the
partials through IPC-mapped mailboxes over xGMI and folds them itself (csrc/include/mireduce/xrank.hpp),
one kernel per step, every device wait bounded; ``rccl`` = a 1-element RCCL all-reduce after the
local kernel (on RCCL's stream); ``auto`` (default) = fused if its self-check passes on every rank,
else rccl. The combine is issued even at N=1 (``--local-only`` skips it), so the 1-GPU run executes
exactly the N-GPU step (at world 1 it exchanges nothing).

Headline = the per-reduction time (reduction.cpp:319-374, mpi/reduce.c:75-79): ONE stream lane,
every step — local reduce AND cross-rank combine — completes before the next starts, replayed from
captured hipGraphs (``--launch``; captured after eager warm-up steps and replayed once untimed:
eager Python issue leaves ~22 us GPU gaps per step). The headline phase runs under a deadline
(``--headline-deadline``): past it rank 0 prints a diagnostic JSON line and every rank exits
non-zero instead of waiting out the process-group timeout. Only after the line is final do the
extras run (pipelined / 2-lane / RCCL candidates, reduce.c's element-wise table, the xGMI peer-read
probe), under their own watchdog (``--extras-deadline``): a hung extra still leaves the printed,
verified headline; the teardown after the line (``--teardown-deadline``) is bounded the same way.
Every step's result is checked after timing against torch's own fp64 reduction
of the shards (AND over ranks), and every device-side error word (polled fan-in, fused finish) is
read and agreed over ranks.

Reference number: 92.7729 GB/s (CUDA DOUBLE SUM, mpi/CUdata.txt:2).
"""
from __future__ import annotations

import argparse
import json
from dataclasses import replace
import math
import os
import signal
import socket
import subprocess
import sys
import time

LAUNCHER_ENV = "MIREDUCE_BENCH_LAUNCHER"  # set by _launch_ranks for its children: "self-spawned"
T0_ENV = "MIREDUCE_BENCH_T0"  # the job's start (time.time()), handed to self-spawned ranks
# The whole run's clock starts here, before torch is imported (a fresh box's first import takes
# minutes): every phase deadline is derived from what is left of --budget.
T0 = float(os.environ.get(T0_ENV) or time.time())
DEFAULT_BUDGET_S = 420.0  # the driver allows 600 s per run; this leaves it a margin
PARENT_GRACE_S = 30.0  # the self-spawning parent kills the ranks this long after the budget


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _no_line(n: int, why: str) -> dict:
    """The diagnostic result line of a run that produced no measurement."""
    return {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": n, "verified": None,
            "higher_is_better": True, "scaling": "strong", "error": why}


def _is_result_line(line: str) -> bool:
    """Whether a relayed stdout line holds a result line — also behind a fragment: a rank's line
    written on the signal path (write(2)) can follow an unterminated piece of Python's buffered
    stdout on the same line."""
    i = line.find("{")
    while i >= 0:
        try:
            d = json.loads(line[i:])
        except ValueError:
            i = line.find("{", i + 1)
            continue
        return isinstance(d, dict) and "metric" in d and "value" in d
    return False


def _relay_child(child, budget_end: float, n: int) -> int:
    """The self-spawning parent's side: relay the ranks' stdout line by line, bound the job at
    ``budget_end`` + PARENT_GRACE_S (SIGTERM to the ranks' process group, SIGKILL 15 s later), and
    if no result line came out, print a diagnostic one itself. Returns the job's exit status."""
    import threading
    seen = {"line": False}

    def pump():
        for raw in iter(child.stdout.readline, b""):
            text = raw.decode("utf-8", "replace")
            if _is_result_line(text.strip()):
                seen["line"] = True
            sys.stdout.write(text)
            sys.stdout.flush()

    th = threading.Thread(target=pump, daemon=True)
    th.start()
    killed = False
    while True:
        try:
            rc = child.wait(timeout=max(0.1, budget_end + PARENT_GRACE_S - time.time()))
            break
        except subprocess.TimeoutExpired:
            killed = True
            print("[bench] the ranks exceeded the run budget: terminating them", file=sys.stderr, flush=True)
            rc = None
            for sig, wait_s in ((signal.SIGTERM, 15.0), (signal.SIGKILL, 15.0)):
                try:
                    os.killpg(child.pid, sig)
                except (ProcessLookupError, PermissionError):
                    pass
                try:
                    rc = child.wait(timeout=wait_s)
                    break
                except subprocess.TimeoutExpired:
                    rc = None
            if rc is None:
                rc = child.wait()
            break
        except KeyboardInterrupt:  # forwarded by the handler; keep waiting for the child's status
            continue
    th.join(timeout=5.0)
    rc = rc if rc >= 0 else 128 - rc  # killed by a signal: the shell's convention
    if not seen["line"]:
        why = ("the ranks exceeded the run budget and were killed" if killed else
               f"the ranks ended (status {rc}) without printing a result line")
        print(json.dumps(_no_line(n, why + "; no measurement")), flush=True)
        return rc if rc != 0 else 2
    return 2 if killed and rc == 0 else rc


def _launch_ranks(argv: list) -> "int | None":
    """Make ``--gpus N`` mean N ranks however bench.py is started. Runs before anything loads the
    HIP runtime (no torch, no native extension): this process never touches a GPU.

    * ``WORLD_SIZE`` set (torchrun / the driver started the ranks): it must equal ``--gpus``, else
      rank 0 prints a diagnostic JSON line and every rank exits with 2 (a mis-launched job must not
      report a 1-rank number as an N-GPU one). Returns None (run the bench in this process).
    * ``WORLD_SIZE`` unset and ``--gpus N > 1``: start ``torch.distributed.run`` with N ranks of this
      same command line as a CHILD process in its own process group (never exec: a replaced process
      image is not allowed on the GPU pool), relay its stdout, forward SIGTERM / SIGINT, enforce the
      run budget on it, print a diagnostic line if it printed none, and return its exit status.
      Each rank records ``launcher: "self-spawned"`` and inherits the job's start time.
    * otherwise (one rank): None.

    Reference: reduce.c reports the rank count it ran with (NODES = commSize, mpi/reduce.c:81,95);
    the job shape comes from the launcher (mpi/ccni_vn.sh:7); every job ends by its wall time
    (mpi/submit_all.sh:4)."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=None)
    pre.add_argument("--budget", type=float, default=DEFAULT_BUDGET_S)
    known, _ = pre.parse_known_args(argv)
    ws = os.environ.get("WORLD_SIZE")
    n = known.gpus if known.gpus is not None else int(ws or 1)  # no --gpus: the launcher's shape
    if ws is not None:
        if int(ws) != n:
            if os.environ.get("RANK", "0") == "0":
                print(json.dumps(_no_line(n, f"--gpus {n} but the launcher started WORLD_SIZE={ws} ranks; "
                                             "refusing to report a measurement for the wrong number of GPUs")),
                      flush=True)
            print(f"[bench] --gpus {n} != WORLD_SIZE {ws}: exiting with 2", file=sys.stderr, flush=True)
            return 2
        return None
    if n <= 1:
        return None
    env = dict(os.environ)
    env[LAUNCHER_ENV] = "self-spawned"
    env[T0_ENV] = repr(T0)
    # the native TCP bootstrap defaults to MASTER_PORT + 17: give it a port known to be free
    env.setdefault("MIREDUCE_BOOTSTRAP_PORT", str(_free_port()))
    master = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(master), os.path.abspath(__file__)] + list(argv)
    print(f"[bench] --gpus {n} without a launcher: starting {n} ranks under torch.distributed.run",
          file=sys.stderr, flush=True)

    def _die_with_parent():  # the child must not outlive a killed parent
        try:
            import ctypes
            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except Exception:  # noqa: BLE001
            pass

    child = subprocess.Popen(cmd, env=env, preexec_fn=_die_with_parent, stdout=subprocess.PIPE,
                             start_new_session=True)

    def _forward(sig, _frame):
        try:
            child.send_signal(sig)
        except ProcessLookupError:
            pass

    for s in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(s, _forward)
    return _relay_child(child, T0 + known.budget, n)


METRIC = "reduction bandwidth (GB/s, whole node), 1B-double sum at 1/2/4/8 MI355X"

if __name__ == "__main__":
    _rc = _launch_ranks(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

import torch  # noqa: E402  (after the launcher: the parent of self-spawned ranks never loads it)

from cuda_mpi_reductions_amd._native import native, native_path  # noqa: E402
from cuda_mpi_reductions_amd.models import CONFIGS, LOC_OPS, NORTH_STAR, scalar_workload  # noqa: E402
from cuda_mpi_reductions_amd.ops import KernelConfig  # noqa: E402
from cuda_mpi_reductions_amd.parallel import dist as pdist  # noqa: E402
from cuda_mpi_reductions_amd.utils.fault import FaultInjector  # noqa: E402
from cuda_mpi_reductions_amd.utils.graphs import StepGraph  # noqa: E402

RELEASE_SETTLE_S = 0.5  # idle after handing GB-sized buffers back to the driver, before timing again


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (ranks) of the job; default: WORLD_SIZE under a launcher, else 1. Without a "
                        "launcher, N > 1 starts N ranks (a child torch.distributed.run)")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default=NORTH_STAR, choices=sorted(CONFIGS))
    p.add_argument("--elements", type=int, default=None, help="override the global element count")
    p.add_argument("--pipelined", action="store_true",
                   help="experiment: a pipelined headline (independent steps overlap: step i+1's local reduce "
                        "with step i's combine, or over --streams lanes) instead of the per-reduction time")
    p.add_argument("--serial", action="store_true", help="(default; kept for old command lines)")
    p.add_argument("--headline-deadline", type=float, default=180.0,
                   help="seconds the headline phase (setup, self-check, plan tuning, timed steps, verification) "
                        "may take; past it rank 0 prints a diagnostic JSON line and every rank exits with 2")
    p.add_argument("--no-candidates", dest="candidates", action="store_false",
                   help="skip the after-headline candidate measurements (pipelined 2-lane fused finish, RCCL "
                        "serial / pipelined)")
    p.add_argument("--collective", choices=["auto", "rccl", "fused"], default="auto",
                   help="cross-rank combine: rccl = 1-element RCCL all-reduce after the local kernel; "
                        "fused = the kernel's last workgroup folds all ranks' partials via IPC mailboxes; "
                        "auto = fused if its self-check passes on every rank, else rccl (GPU scalar configs)")
    p.add_argument("--no-canary", dest="canary", action="store_false",
                   help="at N > 1, skip the fused finish's canary (the same exchange run first in throw-away "
                        "helper processes, so a fault of the peer mapping cannot take the benchmark down)")
    p.add_argument("--canary-timeout", type=float, default=90.0, help="seconds each canary helper may take")
    p.add_argument("--agree-timeout", type=float, default=60.0,
                   help="seconds an optional headline stage (canary verdicts, fused self-check, plan tuning) waits "
                        "for every rank's report; a rank missing past it is dead or hung: rank 0 prints a diagnostic "
                        "line naming the stage and every rank exits with 2 (cut to end before the headline deadline)")
    p.add_argument("--rehearse-stages", action="store_true",
                   help="CPU ranks (--device cpu): also run the GPU-only headline stages in their CPU form — the "
                        "canary (dry helpers), the fused finish's self-check and timed steps over its CPU twin "
                        "(store mailboxes, same timeout semantics) and per-rank plan tuning over the host reducer — "
                        "so their failure boundaries are testable on gloo (tests/test_fault_injection.py)")
    p.add_argument("--xrank-timeout", type=float, default=30.0,
                   help="fused finish: seconds a kernel waits for a peer's partial before flagging the channel")
    p.add_argument("--tune-steps", type=int, default=0,
                   help="--collective auto: steps of the short per-plan measurement that picks the streaming-kernel "
                        "plan (fused finish only); 0 = enough steps for ~30 ms of reduction per plan (20..400)")
    p.add_argument("--vector-impl", choices=["rccl", "direct"], default="rccl",
                   help="vector (reduce.c) configs: torch.distributed collective, or the one-kernel direct "
                        "peer-read collective over xGMI (GPUs)")
    p.add_argument("--no-vector-extras", dest="vector_extras", action="store_false",
                   help="north-star runs also time reduce.c's element-wise table (INT / DOUBLE x MAX / MIN / SUM of "
                        "2 GiB to root 0, plus DOUBLE SUM all-reduce; RCCL and direct) and report it as "
                        "reduce_c_vector; this skips that")
    p.add_argument("--extras-deadline", type=float, default=240.0,
                   help="seconds the reduce.c extras may take after the headline; past it rank 0 prints the "
                        "headline (extras marked as timed out) and the run ends")
    p.add_argument("--teardown-deadline", type=float, default=120.0,
                   help="seconds the teardown after the printed line (device sync, process-group destruction) "
                        "may take; past it every rank exits with the headline's status")
    p.add_argument("--no-decompose", dest="decompose", action="store_false",
                   help="skip the after-headline decomposition (the same steps without the combine, per rank: "
                        "local time, skew, exchange cost)")
    p.add_argument("--local-only", action="store_true",
                   help="single rank: skip the cross-rank combine (by default it is issued even at N=1)")
    p.add_argument("--streams", type=int, default=1,
                   help="with --pipelined: alternate independent steps over this many HIP streams (each with its "
                        "own workspace); the per-reduction headline always runs one lane")
    p.add_argument("--block", type=int, default=0)
    p.add_argument("--unroll", type=int, default=0)
    p.add_argument("--wg-per-cu", type=int, default=0)
    p.add_argument("--policy", choices=["auto", "nt", "default"], default="auto")
    p.add_argument("--no-plan-tune", dest="plan_tune", action="store_false",
                   help="--collective auto on GPUs also measures the streaming-kernel plan for the shard "
                        "(tuned default vs the runners-up, profiles/r2_plan/); this keeps the tuned default")
    p.add_argument("--two-pass", action="store_true")
    p.add_argument("--launch", choices=["auto", "graph", "eager"], default="auto",
                   help="graph: replay the timed steps as captured hipGraphs (chunks of --graph-chunk steps); "
                        "eager: issue every step from Python; auto: graph on GPUs when capturable")
    p.add_argument("--replay-probe", choices=["auto", "on", "off"], default="auto",
                   help="before replaying captured collective-issuing headline steps, replay 3 of them under "
                        "--probe-deadline and fall back to eager issue if any rank fails (auto: when the RCCL "
                        "combine is captured at N > 1)")
    p.add_argument("--probe-deadline", type=float, default=20.0, help="seconds the replay probe may take")
    p.add_argument("--graph-chunk", type=int, default=0,
                   help="steps per captured graph (each graph ends by joining its lanes / last all-reduce, so "
                        "fewer, longer graphs leave fewer bubbles); 0 = auto: every timed step in one graph "
                        "(<= 4096) for the in-kernel fused finish, 128 when steps issue RCCL collectives")
    p.add_argument("--inject-fault", default=None,
                   help="failure-detection test: KIND[@RANK][:STEP][/SITE], KIND = exit|hang|raise|corrupt|delay=<ms>|"
                        "mailbox, SITE = step (headline; steps count warm-up first; forces eager issue) | extras "
                        "(the after-headline candidates) | init | capture | teardown | canary | selfcheck | tune "
                        "(utils/fault.py)")
    p.add_argument("--pg-timeout", type=float, default=120.0, help="process-group collective timeout (s)")
    p.add_argument("--budget", type=float, default=DEFAULT_BUDGET_S,
                   help="seconds the whole run may take, from process start (self-spawned ranks: from the "
                        "parent's start); the headline / extras / teardown deadlines are cut to what is left, "
                        "extras that no longer fit are skipped, and a self-spawning parent kills the ranks "
                        f"{PARENT_GRACE_S:.0f} s past it")
    p.add_argument("--extras-file", default=None,
                   help="where rank 0 writes the full after-headline record (reduce.c table, per-rank plans, "
                        "decomposition, candidates, peer read); default gpurun_out/bench_extras_n<N>.json "
                        "next to bench.py. The printed line carries only the headline and a summary")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--compare-torch", action="store_true",
                   help="after the measurement, time torch's own reduction of the same shard (reported as "
                        "torch_gbps; not part of the metric)")
    p.add_argument("--trace", action="store_true", help="roctx range per step (rocprofv3 --marker-trace)")
    p.add_argument("--backend", choices=["auto", "nccl", "gloo"], default="auto",
                   help="auto: nccl (RCCL) on GPUs, gloo on CPU; gloo + MIREDUCE_FORCE_DEVICE=0 rehearses "
                        "N ranks on one GPU")
    p.add_argument("--device", choices=["auto", "cuda", "cpu"], default="auto",
                   help="cpu: gloo ranks + the native host reducer (tests of the contract only)")
    return p.parse_args(argv)


def _sync(dev: torch.device) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _ranks_seen(ctx) -> int:
    """How many ranks the job's collective backend actually joined: an all-reduce of a one from
    every rank over the default process group (RCCL on GPUs; gloo in CPU rehearsals)."""
    t = torch.ones(1, dtype=torch.int64, device=ctx.device if ctx.backend == "nccl" else "cpu")
    if torch.distributed.is_initialized():
        torch.distributed.all_reduce(t)
    return int(t.item())


def _emit(line: dict) -> bool:
    """Print THE result line (rank 0) through the native once-guard: if a signal handler already
    printed the armed line (the process is being killed), nothing more is printed."""
    sys.stdout.flush()
    return native().emit_final_line(json.dumps(line))


def _arm(line: "dict | None") -> None:
    """The line to print if the process is killed (torchrun SIGTERMs every rank when one fails; a GPU
    fault aborts): csrc/include/mireduce/final_line.hpp. Only rank 0 arms (others pass None)."""
    if line is not None:
        native().arm_final_line(json.dumps(line))


RCCL_KNOBS = ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_BUFFSIZE",
              "NCCL_NTHREADS", "RCCL_MSCCL_ENABLE", "RCCL_MSCCLPP_ENABLE")


def _rccl_env() -> str:
    """The RCCL tuning knobs this run had set ("NCCL_ALGO=Ring NCCL_PROTO=Simple ..."; "" = RCCL's
    defaults): tools/sweep.py --rccl-knobs sweeps them, and the record must say which ran."""
    return " ".join(f"{k}={os.environ[k]}" for k in RCCL_KNOBS if k in os.environ)


def _launch_record(ctx, seen: int) -> dict:
    """JSON fields that prove the job's shape: who started the ranks and how many the collective saw."""
    launcher = os.environ.get(LAUNCHER_ENV) or ("external" if "WORLD_SIZE" in os.environ else "single process")
    return {"launcher": launcher, "ranks_seen": seen, "ranks_seen_backend": ctx.backend,
            "rccl_ranks_seen": seen if ctx.backend == "nccl" else None}


def _time_torch_reduction(wl, K: int, W: int, ctx) -> float:
    """Whole-job GB/s of the same step done with PyTorch's reduction (x.sum / amin / amax on each
    shard, then the same scalar all-reduce) — a vendor-library reference point for the native
    kernel, measured the same way (W warm-up steps, K timed, MAX over ranks)."""
    x, op = wl.x, wl.cfg.op
    acc = wl.acc

    def step():
        if op in LOC_OPS:  # torch.argmax / argmin of the shard, then the same MAXLOC/MINLOC combine
            kind = LOC_OPS[op]
            i = x.argmax() if kind == "max" else x.argmin()
            r = (i + wl.offset).reshape(1)
            if ctx.world_size > 1:
                _, r = pdist.loc_allreduce(x[i].reshape(1), r, kind)
            return r
        if op == "sum":
            r = x.sum(dtype=acc).reshape(1)
        elif op == "sumsq":  # torch's one-pass fused form of the same quantity
            r = torch.linalg.vector_norm(x, 2, dtype=acc).square().reshape(1)
        elif op == "amax":
            r = torch.linalg.vector_norm(x, float("inf")).to(acc).reshape(1)
        else:
            r = (x.amin() if op == "min" else x.amax()).to(acc).reshape(1)
        if ctx.world_size > 1:
            pdist.scalar_allreduce(r, op)
        return r

    for _ in range(W):
        step()
    _sync(ctx.device)
    pdist.barrier(ctx)
    _sync(ctx.device)
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    _sync(ctx.device)
    el = pdist.max_over_ranks(time.perf_counter() - t0, ctx)
    return wl.bytes_total * K / el / 1e9


def _time_vector(wl, ctx, K: int, W: int, fault, verify: bool) -> tuple:
    """Time K element-wise collectives (after W warm-ups), each on its own between a barrier and a
    synchronisation (the in-place buffer is restored outside the clock, like reduce.c's bzero,
    mpi/reduce.c:74-77); returns (sum over steps of the MAX-over-ranks time, verified)."""
    dev = ctx.device
    for i in range(W):
        wl.restore()
        if fault is not None and fault.at(ctx.rank, i, "step", "bench step"):
            wl.corrupt()
        wl.collective()
    times, checks = [], []
    holder = wl.cfg.collective == "allreduce" or ctx.rank == 0
    for i in range(W, W + K):
        wl.restore()
        if fault is not None and fault.at(ctx.rank, i, "step", "bench step"):
            wl.corrupt()  # this rank contributes a wrong element: verification must fail
        _sync(dev)
        pdist.barrier(ctx)
        t0 = time.perf_counter()
        wl.collective()
        _sync(dev)
        times.append(pdist.max_over_ranks(time.perf_counter() - t0, ctx))
        if verify and holder:  # per-step checksum (untimed): every step must agree
            checks.append(wl.result().to(torch.float64).sum().reshape(1))
    verified = None
    if verify:
        same = bool((torch.cat(checks) == checks[-1]).all().item()) if checks else True
        same = -pdist.max_over_ranks(-float(same), ctx) > 0.5  # AND over ranks
        verified = wl.verify()["ok"] and same
    return sum(times), verified


def run_vector(args, ctx, cfg, fault) -> int:
    """reduce.c semantics (BASELINE config 1): element-wise reduce of an N/P vector per rank to
    root 0; the step time is the MAX over ranks; GB = 2^30 B of total data (mpi/reduce.c:79)."""
    from cuda_mpi_reductions_amd.models import VectorReduction
    wl = VectorReduction(cfg, ctx, impl=args.vector_impl).setup(mt19937=(ctx.device.type == "cpu"))
    dev = ctx.device
    elapsed, verified = _time_vector(wl, ctx, args.steps, args.warmup, fault, not args.no_verify)
    gib = wl.bytes_total * args.steps / elapsed / float(1 << 30)
    seen = _ranks_seen(ctx)
    if seen != ctx.world_size:
        verified = False
    if ctx.is_root:
        _emit(({
            "metric": f"MPI_Reduce-style element-wise {cfg.collective} bandwidth (GiB/s of total data, reduce.c units)",
            "value": round(gib, 3), "unit": "GiB/s", "n_gpus": ctx.world_size if dev.type == "cuda" else 0,
            "n_ranks": ctx.world_size, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": round(gib / cfg.baseline, 3) if cfg.baseline else None,
            "dtype": str(cfg.dtype).replace("torch.", ""), "device": dev.type,
            "data": "reduce.c MT19937 per-rank data" if dev.type == "cpu" else "synthetic rank-seeded device fill",
            "config": {"model": f"{cfg.name}: {cfg.description}", "global_batch": wl.count * ctx.world_size,
                       "seq_len": 1, "parallelism": f"dp{ctx.world_size}", "backend": ctx.backend,
                       "impl": wl.impl, "op": cfg.op.upper(), "count_per_rank": wl.count,
                       "rccl_env": _rccl_env()},
            "baseline_value": cfg.baseline, "baseline_unit": cfg.baseline_unit if cfg.baseline else None,
            "baseline_source": cfg.baseline_source or None,
            "verified": verified,
            **_launch_record(ctx, seen),
        }))
    return 0 if verified in (None, True) else 1


REDUCE_C_OPS = ("max", "min", "sum")  # reduce.c's operations[] order = its output row order (reduce.c:26-28)
REDUCE_C_DTYPES = (("INT", "xgmi_2g_int_sum_reduce"), ("DOUBLE", "xgmi_2g_double_sum_reduce"))  # reduce.c:73-97
REDUCE_C_RETRIES = 5  # RETRY_COUNT (mpi/constants.h:5)
REDUCE_C_HEADER = "# DATATYPE OP NODES GB/sec"  # reduce.c:68
WORLD1_RCCL = ("world 1: a 1-rank in-place RCCL reduce enqueues no work (torch.distributed.reduce is in-place), "
               "so there is no number to report; the cross-GPU table needs N > 1")


def _one_collective(wl, ctx) -> float:
    """One timed element-wise collective, as reduce.c times one MPI_Reduce (reduce.c:74-79): the
    receive side is restored outside the clock, then barrier, collective, synchronize; MAX over ranks
    (reduce.c timed on rank 0 only and without a barrier)."""
    wl.restore()
    _sync(ctx.device)
    pdist.barrier(ctx)
    t0 = time.perf_counter()
    wl.collective()
    _sync(ctx.device)
    return pdist.max_over_ranks(time.perf_counter() - t0, ctx)


def _checksum(wl, holder: bool) -> float:
    return float(wl.result().to(torch.float64).sum().item()) if holder else 0.0


def _vector_extras(ctx, retries: int = REDUCE_C_RETRIES, out: "dict | None" = None, progress=None,
                   canary: bool = True, canary_timeout: float = 90.0) -> dict:
    """reduce.c's own measurement on this job's GPUs, next to the scalar headline, in reduce.c's
    shape: element-wise INT and DOUBLE MAX / MIN / SUM of 2 GiB of total data each (NUM_INTS /
    NUM_DOUBLES, mpi/constants.h:1-2) to root 0 (MPI_Reduce, reduce.c:76,90), one warm-up SUM per
    dtype (reduce.c:61-64), then ``retries`` rounds of the six collectives in reduce.c's row order,
    each timed on its own (retry-major, reduce.c:71-97); GiB/s of total data (reduce.c:79,93). Over
    RCCL (torch.distributed, in place: the receive buffer is restored outside the clock like
    reduce.c's bzero) and over the direct one-kernel collective (send buffer -> separate receive
    buffer, like reduce.c's random_* -> reduced_*, reduce.c:46-49).

    ``table``: one entry per timed collective (retry, dtype, op, impl); ``rows``: per impl, exactly
    reduce.c's stdout (header + ``"%s %s %d %10.3lf"`` lines, reduce.c:68,81,95), ready for
    utils/getavgs.py; ``reduce_<impl>`` / ``allreduce_<impl>``: DOUBLE SUM to root / to every rank.
    At world 1 RCCL rows are null (its 1-rank in-place reduce does no work). Every (dtype, op) is
    verified against the gathered inputs on its first retry and later retries must reproduce its
    checksum. Errors are recorded, not raised. ``out`` (optional) is filled in place as the table
    grows, so a watchdog that fires mid-way still reports the rows measured so far; the direct
    collective (no RCCL) goes first."""
    from cuda_mpi_reductions_amd.models import CONFIGS as _C, VectorReduction
    out = {} if out is None else out
    out.update({"units": "GiB/s (2^30 B of total data per collective, reduce.c:93)", "retries": retries,
                "order": "retry-major: per retry INT MAX, INT MIN, INT SUM, DOUBLE MAX, DOUBLE MIN, DOUBLE SUM "
                         "(reduce.c:71-97)", "total_bytes": 256 * 1024 * 1024 * 8})
    # (gloo rehearsals: its GPU-tensor reduce / all_reduce is not RCCL and crashes on 1 GiB
    # tensors, so only the direct collective runs there)
    impls = ("direct", "rccl") if ctx.backend == "nccl" else ("direct",)
    table, rows = [], {}
    out["table"], out["rows"] = table, rows
    holder = ctx.rank == 0
    direct_ok = True
    if ctx.world_size > 1 and canary:  # the peer mapping runs in throw-away helpers first
        from cuda_mpi_reductions_amd.parallel.canary import direct_canary
        why = direct_canary(ctx, timeout_s=canary_timeout)
        if why is not None:
            direct_ok = False
            out["direct_canary"] = why
            impls = tuple(i for i in impls if i != "direct")
            table.append({"impl": "direct", "error": f"canary: {why}"[:300]})
    for impl in impls:
        if impl == "rccl" and ctx.world_size == 1:
            table += [{"dtype": dt, "op": op.upper(), "impl": impl, "gibps": None, "note": WORLD1_RCCL}
                      for dt, _ in REDUCE_C_DTYPES for op in REDUCE_C_OPS]
            out["reduce_rccl"] = out["allreduce_rccl"] = {"gibps": None, "note": WORLD1_RCCL}
            continue
        wls = {}
        lines = [REDUCE_C_HEADER]
        rows[impl] = lines
        try:
            for dt, base in REDUCE_C_DTYPES:  # both registered up front: the rounds interleave dtypes
                wls[dt] = VectorReduction(_C[base], ctx, impl=impl, direct_timeout_s=5.0).setup()
            if impl == "direct" and getattr(wls["DOUBLE"], "comm", None) is not None:
                out["direct_grid"] = wls["DOUBLE"].comm.grid  # CUs / (most ranks sharing one GPU)
            for dt, base in REDUCE_C_DTYPES:  # warm-up SUM per dtype (reduce.c:61-64)
                wls[dt].cfg = replace(_C[base], op="sum")
                _one_collective(wls[dt], ctx)
            first = {}
            for x in range(retries):
                for dt, base in REDUCE_C_DTYPES:
                    wl = wls[dt]
                    for op in REDUCE_C_OPS:
                        wl.cfg = replace(_C[base], op=op)
                        el = _one_collective(wl, ctx)
                        gib = wl.bytes_total / el / float(1 << 30)
                        dev_err = None
                        if x == 0:  # full check against the gathered inputs, and the reference checksum
                            v = wl.verify()
                            ok, dev_err = v["ok"], v.get("device_error")
                            first[(dt, op)] = _checksum(wl, holder)
                        else:
                            same = _checksum(wl, holder) == first[(dt, op)]
                            ok = -pdist.max_over_ranks(-float(same), ctx) > 0.5  # AND over ranks
                        table.append({"retry": x, "dtype": dt, "op": op.upper(), "impl": impl,
                                      "gibps": round(gib, 3), "ms": round(el * 1e3, 4), "verified": ok})
                        if dev_err:
                            table[-1]["device_error"] = dev_err
                        lines.append("%s %s %d %10.3lf" % (dt, op.upper(), ctx.world_size, gib))
                        if progress is not None:
                            progress()  # the rows so far survive a kill of the process
            for kind, coll in (("reduce", "reduce"), ("allreduce", "allreduce")):  # DOUBLE SUM summaries
                wl = wls["DOUBLE"]
                wl.cfg = replace(_C["xgmi_2g_double_sum_reduce"], op="sum", collective=coll)
                els = [_one_collective(wl, ctx) for _ in range(retries)]
                v = wl.verify()
                out[f"{kind}_{impl}"] = {"gibps": round(wl.bytes_total * retries / sum(els) / float(1 << 30), 3),
                                         "ms": round(sum(els) / retries * 1e3, 4), "verified": v["ok"]}
                if v.get("device_error"):
                    out[f"{kind}_{impl}"]["device_error"] = v["device_error"]
        except Exception as e:  # noqa: BLE001 - an extra must never cost the headline
            import traceback
            err = {"error": f"{type(e).__name__}: {e}"[:200]}
            print(f"[bench] rank {ctx.rank}: reduce.c extra ({impl}) failed:\n{traceback.format_exc()}",
                  file=sys.stderr)
            table.append({"impl": impl, **err})
            out.setdefault(f"reduce_{impl}", err)
            out.setdefault(f"allreduce_{impl}", err)
        for wl in wls.values():
            wl.close()  # collective: the next registration may reuse these addresses
        wls.clear()
        torch.cuda.empty_cache()
        # GB-sized buffers just went back to the driver: the stream that follows such a release runs
        # ~6 % slow for a few tens of ms (profiles/r3_passW/settle_bf16.txt, phases E and G), so the
        # next measurement starts after it has passed.
        time.sleep(RELEASE_SETTLE_S)
    if ctx.world_size == 1:
        out["note"] = ("world 1: RCCL rows are null (no work); direct is one local send -> receive pass (what "
                       "MPI_Reduce does on one rank); tools/scaling.py keeps N=1 out of the results files")
    if ctx.world_size > 1:
        out["peer_read"] = _peer_read_extra(ctx) if direct_ok else {"error": "skipped: the direct canary failed"}
    return out


def _auto_tune_steps(bytes_per_gpu: float, target_s: float = 0.03) -> int:
    """Tuning steps per candidate: ~``target_s`` of reduction at ~7 TB/s per GPU (20 steps of a
    1 GB shard are 2.8 ms — within launch noise of each other), clamped to 20..400."""
    return int(min(400, max(20, math.ceil(target_s / max(bytes_per_gpu / 7e12, 1e-9)))))


def _peer_read_extra(ctx, nbytes: int = 256 << 20, steps: int = 5) -> dict:
    """xGMI ingress roofline on this job's GPUs (bandwidth_test --peer, simpleP2P.cu:314-329): every
    rank's one-kernel read of ``nbytes`` from each of its world-1 peers at once, all ranks together
    (between barriers). Per-rank ingress GB/s (min / max over ranks) and the node aggregate (all
    bytes moved / the slowest rank's time). Errors are recorded, not raised."""
    from cuda_mpi_reductions_amd.parallel import DirectComm
    dev, world = ctx.device, ctx.world_size
    try:
        comm = DirectComm(dev, nbytes, timeout_s=5.0)  # collective: fails on every rank together
    except Exception as e:  # noqa: BLE001 - an extra must never cost the headline
        return {"error": f"{type(e).__name__}: {e}"[:400]}
    err, el = None, float("inf")
    try:
        comm.read_peers(nbytes)  # warm-up (maps, TLB)
        _sync(dev)
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"[:200]
    pdist.barrier(ctx)  # every rank reaches every collective below, failed or not
    if err is None:
        try:
            t0 = time.perf_counter()
            for _ in range(steps):
                comm.read_peers(nbytes)
            _sync(dev)
            el = time.perf_counter() - t0
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"[:200]
    failed = pdist.max_over_ranks(1.0 if err else 0.0, ctx) > 0.5
    ingress = 0.0 if err else (world - 1) * nbytes * steps / el / 1e9
    lo = -pdist.max_over_ranks(-ingress, ctx)
    hi = pdist.max_over_ranks(ingress, ctx)
    slowest = pdist.max_over_ranks(el if not err else 0.0, ctx)
    comm.close()
    if failed:
        errs = [None] * world
        torch.distributed.all_gather_object(errs, err)
        return {"error": "; ".join(f"rank {r}: {m}" for r, m in enumerate(errs) if m)[:400]}
    return {"bytes_per_peer": nbytes, "steps": steps, "ingress_gbps_min": round(lo, 2),
            "ingress_gbps_max": round(hi, 2),
            "node_gbps": round(world * (world - 1) * nbytes * steps / slowest / 1e9, 2)}


def _plan_candidates(bytes_per_gpu: float, esize: int) -> list:
    """Streaming-kernel plans (block, unroll, workgroups per CU, load window, XCD skew) worth
    measuring on the node for a shard of this size: (0, 0, 0, -1, None) = the tuned default
    (256x8x1 with an explicit load window of 4 and the XCD-weighted split for 8-byte types above
    192 MB, profiles/r3_window/, profiles/r4_xcd/). The ranking of the top plans moves by 1-2 %
    between boxes, so for the headline's 8-byte shards the bench measures the default against the
    same plan with equal rounds per XCD (skew 0), with twice the skew, with the skew favouring the
    EVEN XCCs (-20: a GPU whose even XCDs are the faster half) and against the runner-up of the
    round-3 window sweep, instead of trusting one box's table. Each rank keeps its own best
    (_tune_plan)."""
    if esize == 8 and bytes_per_gpu >= 768 * (1 << 20):
        return [(0, 0, 0, -1, None), (0, 0, 0, -1, 0), (0, 0, 0, -1, 40), (0, 0, 0, -1, -20), (256, 4, 2, 2, None)]
    return [(0, 0, 0, -1, None)]


def _plan_key(c) -> str:
    b, u, w, win, skew = c
    if b == 0:
        return "tuned default" + ("" if skew is None else f", XCD skew {skew}")
    return f"{b}x{u}x{w}" + (f" window {win}" if win > 0 else " hipcc schedule") + \
        ("" if skew is None else f", XCD skew {skew}")


def _graph_chunk(requested: int, steps: int, issues_collective: bool) -> int:
    """Steps per captured graph. Auto: one graph for all the steps when they are kernels only (the
    fused finish; measured at the 1 GB N=8 shard with 2 lanes, 1000 steps: 7.32-7.34 TB/s as one
    graph vs 7.17-7.27 in chunks of 128, profiles/r2_shard/run4.sh), 128 when every step also
    captures an RCCL collective."""
    if requested > 0:
        return requested
    return 128 if issues_collective else max(1, min(steps, 4096))


def _measure(wl, slots, ctx, args, fault, serial: bool, warmup: int, allow_graph: bool = True,
             steps: "int | None" = None, site: str = "step", step_fn=None) -> dict:
    """Time K steps (after ``warmup`` eager steps); returns elapsed (MAX over ranks; ``elapsed_min``:
    the fastest rank's), the launch mode and how many slots the timed steps wrote (graph replays
    rewrite the first chunk). ``site``: the fault-injection site of these steps (``step`` = the
    headline, ``extras`` = a candidate). ``step_fn`` (default ``wl.step``): what one step enqueues."""
    C = native()
    dev = ctx.device
    K = args.steps if steps is None else steps
    step = step_fn or wl.step
    issues_collective = wl.issues_collective and step_fn is None

    def run(first: int, count: int):
        works = []
        wl.fork()
        for i in range(first, first + count):
            C.trace_push("bench.step")
            corrupt = fault.at(ctx.rank, i, site, f"bench {site}")
            w = step(slots[i:i + 1], async_op=True, corrupt=corrupt)
            C.trace_pop()
            if w is not None:
                if serial:
                    w.wait()
                else:
                    works.append(w)
        for w in works:
            w.wait()
        wl.join()

    run(0, warmup)
    launch, sg = "eager", None
    armed = fault.on(site)
    capturable = dev.type == "cuda" and not args.trace and not armed and \
        (not issues_collective or ctx.backend == "nccl")
    # The headline's captured collectives get a short replay probe first (--replay-probe)
    probe = site == "step" and (args.replay_probe == "on" or (
        args.replay_probe == "auto" and issues_collective and ctx.world_size > 1))
    if allow_graph and ((args.launch == "graph" and not armed) or (args.launch == "auto" and capturable)):
        # Capture the K timed steps as graph replays of --graph-chunk-step chunks (all ranks agree
        # on success or all fall back to eager issue); one untimed replay uploads the graphs.
        W = warmup
        sg = StepGraph(lambda j: step(slots[W + j:W + j + 1], async_op=True), K, dev,
                       chunk=_graph_chunk(args.graph_chunk, K, issues_collective), serial=serial,
                       fork=wl.fork, join=wl.join)
        # (kernel-only steps keep the NCCL stream out of the capture: no watchdog settle needed)
        if sg.capture(group_agree=ctx.world_size > 1, settle_s=None if issues_collective else 0.0):
            launch = f"graph (chunk {sg.chunk}, {sg.reps} replays" + (f" + 1 of {sg.rem})" if sg.rem else ")")
            perr = _replay_probe(wl, ctx, args, fault, serial, step, capture=True) if probe else None
            if perr is not None:
                sg.reset()
                sg = None
                launch = f"eager (captured replay probe failed: {perr})"
                if ctx.is_root:
                    print(f"[bench] {launch}", file=sys.stderr)
            else:
                if probe:
                    launch += "; replay probe ok"
                for g in sg.graphs:
                    g.replay()
        else:
            launch = f"eager (graph capture failed: {sg.error})"
            if ctx.is_root:
                print(f"[bench] {launch}", file=sys.stderr)
            sg = None
    elif probe:  # no graphs here (CPU rehearsal, --launch eager): the same probe over eager steps
        perr = _replay_probe(wl, ctx, args, fault, serial, step, capture=False)
        launch = f"eager (replay probe failed: {perr})" if perr else "eager; replay probe ok"
    probe_window = os.environ.get("MIREDUCE_WINDOW_PROBE") == "1" and dev.type == "cuda"  # diagnostic
    _sync(dev)
    pdist.barrier(ctx)
    _sync(dev)
    if probe_window:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    if probe_window:
        ev[0].record()
    if sg is not None:
        sg.run()
    else:
        run(warmup, K)
    if probe_window:
        ev[1].record()
        t_enq = time.perf_counter()
    _sync(dev)
    t1 = time.perf_counter()
    if probe_window:
        gpu = ev[0].elapsed_time(ev[1]) * 1e-3
        print(f"[window] rank {ctx.rank} site {site} K {K}: host {(t1 - t0) * 1e6:.1f} us, gpu {gpu * 1e6:.1f} us, "
              f"enqueue {(t_enq - t0) * 1e6:.1f} us, host - gpu {(t1 - t0 - gpu) * 1e6:.1f} us", file=sys.stderr)
    pdist.barrier(ctx)
    elapsed = pdist.max_over_ranks(t1 - t0, ctx)
    fastest = -pdist.max_over_ranks(-(t1 - t0), ctx)
    written = warmup + (sg.chunk if sg is not None else K)
    if sg is not None:
        sg.reset()  # captured RCCL work must not outlive the communicator
    return {"elapsed": elapsed, "elapsed_min": fastest, "elapsed_local": t1 - t0, "launch": launch,
            "written": written}


def _replay_probe(wl, ctx, args, fault, serial: bool, step, capture: bool) -> "str | None":
    """Before the headline replays captured collective-issuing steps (the RCCL combine at N > 1,
    used when the fused finish was declined): capture 3 such steps, replay them once and poll for
    completion for at most ``--probe-deadline`` seconds; the verdict is agreed over ranks. Any
    failure (capture error, replay error, late completion on any rank) makes the headline issue its
    steps eagerly, and the JSON's ``launch`` says why — a problem of the captured path must not cost
    the number. A replay that NEVER completes cannot be recovered in-process (its stream is stuck
    behind a spinning collective kernel): the headline deadline then ends the run with rc 2 and a
    diagnostic line. Without graphs (``capture=False``: CPU rehearsals) 3 eager steps are probed
    under the same rules. Fault site ``capture`` (STEP ignored) fires inside the probe's clock.
    Reference: every reduction is timed to completion and none may be lost (reduction.cpp:319-374)."""
    dev = ctx.device
    deadline = args.probe_deadline
    slots = wl.new_slots(3)
    err, pg, done = None, None, True
    try:
        if capture:
            pg = StepGraph(lambda j: step(slots[j:j + 1], async_op=True), 3, dev, chunk=3, serial=serial,
                           fork=wl.fork, join=wl.join)
            if not pg.capture(group_agree=ctx.world_size > 1):
                err, pg = f"capture: {pg.error}", None
        if err is None:
            t0 = time.perf_counter()
            fault.at(ctx.rank, fault.spec.step, "capture", "replay probe")
            if pg is not None:
                pg.run()
                ev = torch.cuda.Event()
                ev.record()
                while not ev.query() and time.perf_counter() - t0 <= deadline:
                    time.sleep(0.0005)
                done = ev.query()
            else:
                for j in range(3):
                    w = step(slots[j:j + 1], async_op=True)
                    if w is not None:
                        w.wait()
                _sync(dev)
            el = time.perf_counter() - t0
            if not done:
                err = f"3 replayed steps not complete after {deadline:g} s"
            elif el > deadline:
                err = f"3 steps took {el:.1f} s (deadline {deadline:g} s)"
    except Exception as e:  # noqa: BLE001 - recorded; the headline falls back to eager issue
        err = f"{type(e).__name__}: {e}"[:200]
    failed = pdist.max_over_ranks(1.0 if err else 0.0, ctx) > 0.5  # (waits for a stuck rank's stream)
    if pg is not None:
        _sync(dev)
        pg.reset()
    if not failed:
        return None
    errs = [err]
    if ctx.world_size > 1:
        errs = [None] * ctx.world_size
        torch.distributed.all_gather_object(errs, err)
    return "; ".join(f"rank {r}: {m}" for r, m in enumerate(errs) if m)[:300] or "failed on another rank"


def _agree_timeout(args, at_least: float = 0.0) -> float:
    """The bound of an optional stage's agreement: --agree-timeout (or ``at_least``, the longest a
    live rank can legitimately take to arrive: a fused step waits up to --xrank-timeout for a peer
    that failed before launching), cut so that a lost rank is reported by the agreement (its stage
    named) before the headline deadline would fire."""
    want = max(args.agree_timeout, at_least)
    left = getattr(args, "_headline_ends", None)
    cap = (left - time.time() - 5.0) if left else want
    return max(1.0, min(want, cap))


def _try_fused(wl, ctx, args, fault, at_stage=lambda name: None) -> "str | None":
    """Switch the workload to the fused in-kernel finish and check it on every rank; on any failure
    switch back to RCCL (every rank together) and return the reason. Three stages, each behind a
    failure boundary agreed over ranks (an optional 0.5 % path must never cost
    the one-shot N-GPU measurement):

    * ``canary`` (N > 1): the same exchange in throw-away helper processes first
      (parallel/canary.py) — a fault of the peer mapping there cannot take this process, and the
      headline, down with it; the helpers' verdicts are agreed through a bounded store exchange;
    * channel setup: collective by construction (``open_channel`` raises on every rank together);
    * ``fused self-check``: one bounded agreement that every rank is ready (a rank that failed
      before launching makes every rank fall back at once, not after a peer's fused step waited
      --xrank-timeout for it); then 3 fused steps, this rank's error words and the same kernel's
      partial without a channel — all LOCAL, inside a try — then one bounded agreement
      (:func:`parallel.dist.agree`) of every rank's report, from which every rank derives the same
      verdict. A rank whose part raised reports the error; one that died or hangs makes the others
      raise :class:`parallel.dist.PeerLost` (main() prints the diagnostic line naming the stage)
      instead of waiting in a collective until the process-group timeout.

    Fault sites ``canary`` / ``selfcheck`` (utils/fault.py) fire inside these stages."""
    if args.canary and ctx.world_size > 1:
        at_stage("canary")
        from cuda_mpi_reductions_amd.parallel.canary import fused_canary
        # (a rank whose helper failed at once arrives up to --canary-timeout before one whose helper
        # waited the full timeout for it: the bound outlasts that)
        err = fused_canary(ctx, timeout_s=args.canary_timeout, dry=ctx.device.type != "cuda", fault=fault,
                           agree_timeout_s=_agree_timeout(args, args.canary_timeout + 10.0))
        if err is not None:
            return f"canary: {err}"[:300]
    at_stage("fused self-check")
    try:
        wl.use_collective("fused", streams=1)  # collective; raises on every rank if any rank cannot map
    except Exception as e:  # noqa: BLE001
        wl.use_collective("rccl", streams=1)
        return f"setup: {e}"[:300]
    mine = {"error": None}

    def failed_here(e: Exception) -> None:
        mine["error"] = f"{type(e).__name__}: {e}"[:200]
        print(f"[bench] rank {ctx.rank}: fused self-check failed here: {mine['error']}", file=sys.stderr, flush=True)
    try:
        fault.at(ctx.rank, fault.spec.step, "selfcheck", "fused self-check")
        slots = wl.new_slots(3)
    except Exception as e:  # noqa: BLE001 - this rank's report carries it; every rank falls back together
        failed_here(e)
    # Every rank ready before any fused launch: a rank that failed before its steps would otherwise
    # leave the others' first fused step waiting --xrank-timeout in the kernel for its partial.
    ready = pdist.agree(ctx, "fused self-check", {"error": mine["error"]}, _agree_timeout(args))
    errs = [f"rank {r}: {row['error']}" for r, row in enumerate(ready) if row.get("error")]
    if errs:
        wl.use_collective("rccl", streams=1)
        return ("self-check: " + "; ".join(errs))[:300]
    try:
        for i in range(3):
            wl.step(slots[i:i + 1])
        mine.update(_selfcheck_report(wl, slots))
    except Exception as e:  # noqa: BLE001 - as above
        failed_here(e)
    # (a rank that fails during its steps still makes the others' fused steps wait --xrank-timeout)
    rows = pdist.agree(ctx, "fused self-check", mine, _agree_timeout(args, args.xrank_timeout + 10.0))
    if (mine.get("counts") or [0])[0]:
        wl.reset_fanin()  # this rank's sticky fan-in error was reported: clear it
    ok, ref = _selfcheck_verdict(rows, wl.cfg.op, wl.new_slots(1).dtype)
    if ok:
        return None
    wl.use_collective("rccl", streams=1)  # every rank: the verdict is the same everywhere
    return ref["reason"][:300]


def _py(v):
    """A tensor element as a JSON-exact Python number (float repr round-trips; ints are exact)."""
    return float(v) if isinstance(v, float) else int(v)


def _selfcheck_report(wl, slots: torch.Tensor) -> dict:
    """This rank's part of the fused self-check, local only: its error words (the fused finish's
    and the fan-in's), the SAME kernel's partial launched without a channel (what the exchange
    combines), and the slots the fused steps wrote."""
    loc = wl.new_slots(1)
    wl.local(loc)
    if loc.is_cuda:
        torch.cuda.synchronize(loc.device)
    counts = wl.error_counts() if hasattr(wl, "error_counts") else [0, 0, 0, 0]
    p = _py(loc.cpu().item())
    return {"counts": counts, "partial": p, "mag": abs(float(p)), "slots": [_py(v) for v in slots.cpu().tolist()]}


def _selfcheck_verdict(rows: list, op: str, acc: torch.dtype) -> tuple:
    """(ok, ref) from every rank's :func:`_selfcheck_report` (the same on every rank): any rank's
    error, any device error word, or any slot that differs from the fold of the ranks' channel-free
    partials fails it — exactly for MIN/MAX and integers, within a few ulps of the accumulator for
    floating SUM (the partials fold in another order)."""
    errs = [f"rank {r}: {row['error']}" for r, row in enumerate(rows) if row.get("error")]
    if errs:
        return False, {"reason": "self-check: " + "; ".join(errs)}
    from cuda_mpi_reductions_amd.models import ScalarReduction
    counts = [sum(int(row["counts"][k]) for row in rows) for k in range(4)]
    dev_err = ScalarReduction.describe_errors(counts)
    if dev_err:
        return False, {"reason": dev_err}
    parts = [row["partial"] for row in rows]
    if op in ("min",):
        expect = min(parts)
    elif op in ("max", "amax"):
        expect = max(parts)
    else:
        expect = parts[0]
        for v in parts[1:]:
            expect = expect + v
    floating = acc.is_floating_point
    tol = 0.0
    if floating and op in ("sum", "sumsq"):
        tol = 8.0 * len(rows) * torch.finfo(acc).eps * sum(row["mag"] for row in rows)
    bad = []
    for r, row in enumerate(rows):
        for v in row["slots"]:
            if floating:
                if not abs(float(v) - float(expect)) <= tol:  # (NaN: never within)
                    bad.append((r, v))
            elif int(v) != int(expect):
                bad.append((r, v))
    ref = {"got": rows[0]["slots"], "expected": expect, "tolerance": tol}
    if bad:
        ref["reason"] = f"self-check mismatch: {ref} (rank, slot) {bad[:4]}"
        return False, ref
    return True, ref


def _selfcheck_slots(wl, slots: torch.Tensor, ctx, timeout_s: float = 60.0) -> tuple:
    """The fused finish's self-check value: this rank's partial from the SAME kernel launched
    without a channel, combined over the ranks (what the fused exchange replaces). It tests the
    exchange, not the kernel, and needs no torch pass over the array before the timed steps: the
    full torch reference still checks every timed slot afterwards (``_verify_slots``). Every slot
    must match on every rank; the reports are agreed through one bounded store exchange."""
    rows = pdist.agree(ctx, "fused self-check", _selfcheck_report(wl, slots), timeout_s)
    return _selfcheck_verdict(rows, wl.cfg.op, slots.dtype)


def _verify_slots(wl, written: torch.Tensor, ctx) -> tuple:
    """Every slot must hold the global value (all steps reduce the same data); AND over ranks."""
    ref = wl.verify(written[-1:])
    ok = ref["ok"]
    if written.numel() > 1:
        s = written
        if wl.cfg.op in ("sum", "sumsq") and s.dtype.is_floating_point:
            ok = ok and bool(((s - s[-1]).abs() <= ref["tolerance"]).all().item())
        else:
            ok = ok and bool((s == s[-1]).all().item())
    ok = -pdist.max_over_ranks(-float(ok), ctx) > 0.5
    return ok, ref


class _PhaseWatchdog:
    """Deadline for one phase of the run. If it passes first, rank 0 prints ``make_line()`` (when
    not None) and every rank exits with ``rc``: a phase hung in a collective (e.g. one rank failing
    inside it while the others wait) must not hold the run until the process-group timeout."""

    def __init__(self, what: str, deadline_s: float, rc: int, make_line):
        import threading
        self._what, self._deadline, self._rc, self._make_line = what, deadline_s, rc, make_line
        self._lock = threading.Lock()
        self._done = False
        self._timer = threading.Timer(deadline_s, self._fire)
        self._timer.daemon = True
        self._timer.start()

    def _fire(self) -> None:
        with self._lock:
            if self._done:
                return
            self._done = True
            line = self._make_line()
            if line is not None:
                _emit(line)
            print(f"[bench] {self._what} exceeded {self._deadline:.0f} s: exiting with {self._rc}",
                  file=sys.stderr, flush=True)
            os._exit(self._rc)

    def finish(self) -> bool:
        """True if the phase finished before the deadline (the caller goes on)."""
        with self._lock:
            self._timer.cancel()
            if self._done:
                return False
            self._done = True
            return True


def _collect_verified(obj, out: list) -> list:
    """Every ``verified`` flag (not None) anywhere in an extras record."""
    if isinstance(obj, dict):
        for k, v in obj.items():
            if k == "verified" and v is not None:
                out.append(bool(v))
            else:
                _collect_verified(v, out)
    elif isinstance(obj, list):
        for v in obj:
            _collect_verified(v, out)
    return out


def _reduce_c_means(table: list) -> dict:
    """reduce.c's table as the driver's record can keep it: per impl, one ``"DATATYPE OP GiB/s"``
    row per collective in reduce.c's order, averaged over the retries the way getAvgs.sh averages
    each results file (mpi/getAvgs.sh:3-14, reduce.c:71-97); a row with an unverified retry is
    marked ``!``. NODES is the line's ``n_gpus``."""
    acc: dict = {}
    for t in table:
        if not isinstance(t, dict) or t.get("gibps") is None or "dtype" not in t:
            continue
        e = acc.setdefault(t["impl"], {}).setdefault((t["dtype"], t["op"]), [0.0, 0, True])
        e[0] += float(t["gibps"])
        e[1] += 1
        e[2] = e[2] and t.get("verified") is not False
    return {impl: "; ".join(f"{dt} {op} {tot / n:.3f}" + ("" if ok else "!") for (dt, op), (tot, n, ok) in rows.items())
            for impl, rows in acc.items()}


def _summarise(ex: dict) -> dict:
    """The few extras numbers the printed line carries (the full record is the sidecar)."""
    s = {}
    pt = ex.get("plan_tuning")
    if isinstance(pt, dict) and pt.get("plan_by_rank"):
        s["plans"] = _plans_summary(pt["plan_by_rank"])
    c = ex.get("candidates")
    if isinstance(c, dict):
        pipe = [v["gbps"] for k, v in c.items() if k.endswith("pipelined") and isinstance(v, dict) and v.get("gbps")]
        s["pipelined_gbps"] = max(pipe) if pipe else None
        s["rccl_serial_gbps"] = (c.get("rccl_serial") or {}).get("gbps")
    dec = ex.get("decomposition")
    if isinstance(dec, dict) and "error" not in dec:
        s["local_gbps"] = dec.get("local_gbps")
        s["efficiency_vs_local"] = dec.get("scaling_efficiency_vs_local")
        s["exchange_us"] = dec.get("exchange_us_per_step")
        if dec.get("skew_us_per_step") is not None:
            s["skew_us"] = dec["skew_us_per_step"]
        w = dec.get("exchange_wait_us")
        if isinstance(w, dict) and w.get("min_rank_median") is not None:  # device-timed push -> all partials
            s["wait_us"] = [w["min_rank_median"], w["max_rank_median"]]
    v = ex.get("reduce_c_vector")
    if isinstance(v, dict):
        s["reduce_c_gibps"] = {impl: (v.get(f"reduce_{impl}") or {}).get("gibps") for impl in ("direct", "rccl")}
        means = _reduce_c_means(v.get("table") or [])
        if means:
            s["reduce_c_rows"] = means
        if isinstance(v.get("peer_read"), dict):
            s["peer_node_gbps"] = v["peer_read"].get("node_gbps")
    if "torch_gbps" in ex:
        s["torch_gbps"] = ex["torch_gbps"]
    if "skipped" in ex:
        s["extras_skipped"] = ex["skipped"]
    flags = _collect_verified(ex, [])
    s["extras_verified"] = all(flags) if flags else None
    return s


EXTRAS_DIR_ENV = "MIREDUCE_EXTRAS_DIR"  # where the default sidecar goes (the tests give each run its own)


def _default_extras_path(n: int) -> str:
    d = os.environ.get(EXTRAS_DIR_ENV) or os.path.join(os.path.dirname(os.path.abspath(__file__)), "gpurun_out")
    return os.path.join(d, f"bench_extras_n{n}.json")


class _Record:
    """Rank 0's result. The printed line is compact and self-proving: the driver contract's keys,
    ``verified`` / ``ranks_seen`` / ``rccl_ranks_seen`` among the first, the launcher and the
    native source hash, and a small ``summary`` of the extras. Everything else — the long config
    descriptions, the kernel plan, the topology, the per-rank plan tuning, the decomposition, the
    candidates, reduce.c's whole table, the peer read — goes to a JSON sidecar (``path``), written
    again at every update so a killed run still leaves what it measured. The sidecar holds the line
    merged with all of it (tools/scaling.py reads either). Reference: reduce.c prints one short
    row per measurement (mpi/reduce.c:81,95)."""

    def __init__(self, line: dict, detail: dict, path: str):
        import threading
        self.line, self.detail, self.path = line, detail, path
        self.extras: dict = {}
        self.run = f"{int(time.time() * 1e3):x}-{os.getpid():x}"
        self._lock = threading.Lock()  # the extras watchdog's thread may write while the main thread does

    def _snapshot(self) -> dict:
        for _ in range(5):  # the extras may be mid-update in the main thread: snapshot via JSON
            try:
                return json.loads(json.dumps(self.extras))
            except (RuntimeError, ValueError):
                time.sleep(0.01)
        return {}

    def final(self, error: "str | None" = None) -> dict:
        """The line to print (and the sidecar, written as a side effect). ``error``: why the
        extras stopped early (they are then marked so in the sidecar)."""
        ex = self._snapshot()
        if error and isinstance(ex.get("reduce_c_vector"), dict):
            ex["reduce_c_vector"]["error"] = error
        summary = _summarise(ex)
        summary["run"] = self.run
        if error:
            summary["extras_error"] = error
        summary["extras_file"] = self.path
        out = dict(self.line)
        out["summary"] = summary
        try:
            with self._lock:
                os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
                tmp = f"{self.path}.{os.getpid()}.tmp"
                with open(tmp, "w") as f:
                    json.dump({**out, **self.detail, **ex}, f, indent=1)
                os.replace(tmp, self.path)
        except (OSError, TypeError, ValueError) as e:  # the line must still print
            summary["extras_file"] = None
            summary["extras_file_error"] = f"{type(e).__name__}: {e}"[:160]
        return out


class _ExtrasWatchdog(_PhaseWatchdog):
    """The after-headline extras' deadline: on expiry the finished headline is printed with the
    summary of whatever extras completed so far (the record's sidecar keeps them all, the rest
    marked as timed out), and every rank exits with the headline's status."""

    def __init__(self, record: "_Record | None", deadline_s: float, rc: int):
        msg = f"extras did not finish within {deadline_s:.0f} s (headline measured and verified before them)"
        super().__init__("after-headline extras", deadline_s, rc,
                         lambda: record.final(error=msg) if record is not None else None)


def _gbps(wl, K: int, elapsed: float) -> float:
    return wl.bytes_total * K / elapsed / 1e9


def _candidates(wl, ctx, args, fault, fused_ok: bool, capture_failed: bool = False, which: str = "all") -> dict:
    """After-headline measurements of the other step protocols (extras; never the headline):

    * ``fused_2lane_pipelined``: the fused finish over two stream lanes, consecutive independent
      reductions overlapping (one step's tail with the next one's body);
    * ``rccl_serial`` / ``rccl_pipelined``: the 1-element RCCL all-reduce combine, each step to
      completion / the all-reduce of step i overlapping the local reduce of step i+1 (N > 1 only:
      at world 1 the all-reduce enqueues no kernel).

    ``which``: ``fused`` / ``rccl`` / ``all`` of them. Each one's error words are read right after
    it; the slots of all of them are verified after the last measurement (a torch reference pass
    slows the run that follows it, ``profiles/r3_selfcheck/``). A failure is recorded, never raised. Fault site
    ``extras`` injects into these steps. ``capture_failed``: the headline's graph capture of
    collective-issuing steps failed (e.g. gloo collectives on GPU tensors), so RCCL candidates are
    issued eagerly rather than captured again (a second failed capture can abort the process)."""
    K, W = args.steps, min(args.warmup, 2)
    todo = []
    if fused_ok and which in ("all", "fused"):
        todo.append(("fused_2lane_pipelined", "fused", 2, False))
    if ctx.world_size > 1 and which in ("all", "rccl"):
        todo += [("rccl_serial", "rccl", 1, True), ("rccl_pipelined", "rccl", 1, False)]
    out = {}
    pending = []  # verified after ALL candidates are measured: a torch pass slows the run after it
    for name, coll, lanes, serial in todo:
        try:
            wl.use_collective(coll, streams=lanes)
            slots = wl.new_slots(W + K)
            m = _measure(wl, slots, ctx, args, fault, serial=serial, warmup=W, site="extras",
                         allow_graph=not (capture_failed and coll == "rccl"))
            err = wl.check()
            out[name] = {"gbps": round(_gbps(wl, K, m["elapsed"]), 3),
                         "ms_per_step": round(m["elapsed"] / K * 1e3, 5), "launch": m["launch"], "verified": None}
            if err:
                out[name]["error"] = err
            pending.append((name, slots[:m["written"]]))
        except Exception as e:  # noqa: BLE001 - an extra must never cost the headline
            out[name] = {"error": f"{type(e).__name__}: {e}"[:300]}
            print(f"[bench] rank {ctx.rank}: candidate {name} failed: {e}", file=sys.stderr)
    for name, written in pending:
        try:
            out[name]["verified"] = _verify_slots(wl, written, ctx)[0] and "error" not in out[name]
        except Exception as e:  # noqa: BLE001
            out[name].update(verified=False, error=f"verification: {type(e).__name__}: {e}"[:300])
    if ctx.world_size == 1 and which in ("all", "rccl"):
        out["rccl_serial"] = out["rccl_pipelined"] = {"gbps": None, "note": "world 1: a 1-rank RCCL all-reduce "
                                                      "enqueues no kernel, so there is no combine to measure"}
    return out


def _decompose(wl, ctx, args, fault, headline_ms: float, allow_graph: bool = True) -> dict:
    """Where the N-GPU step's time goes (an extra, measured after the line is final): the same
    serial, graph-replayed steps with the combine removed (``wl.local_step``: the same kernel plan,
    no channel, no collective), timed per rank.

    * ``local_ms_per_step``: the slowest rank's local time per step (= ``local_ms_max``);
      ``local_ms_min``: the fastest rank's; their difference is the inter-GPU skew of the local work;
    * ``local_gbps``: bytes per step / slowest local time (the node rate if combining were free);
    * ``exchange_us_per_step``: headline ms/step - slowest local ms/step: the cross-rank combine's
      round trip plus the per-step skew it exposes (each combine waits for the slowest rank);
    * ``scaling_efficiency_vs_local``: value / (N x the slowest rank's local rate) — how much of the
      local reduction rate survives the combine (1.0 = combining is free). Not the N-vs-1 scaling
      efficiency, which tools/scaling.py computes from the per-N headline values.

    Reference shape: whole-node GB/s = bytes / max over ranks (t_local + t_combine) (SURVEY §5.8;
    simpleMPI.cpp:92-98: local reduce, then the combine)."""
    K, W = args.steps, min(args.warmup, 2)
    slots = wl.new_slots(W + K)
    m = _measure(wl, slots, ctx, args, fault, serial=True, warmup=W, site="extras", step_fn=wl.local_step,
                 allow_graph=allow_graph)
    written = slots[:m["written"]]
    same = bool((written == written[-1]).all().item()) if written.numel() else True
    same = -pdist.max_over_ranks(-float(same), ctx) > 0.5  # every slot holds this rank's partial
    err = wl.check()
    wait = _exchange_wait(wl, ctx, args, fault, allow_graph=allow_graph) \
        if getattr(wl, "collective", None) == "fused" and wl.channels else None
    loc_max, loc_min = m["elapsed"] / K * 1e3, m["elapsed_min"] / K * 1e3
    out = {"local_ms_per_step": round(loc_max, 5), "local_ms_min": round(loc_min, 5), "local_ms_max": round(loc_max, 5),
           "local_gbps": round(wl.bytes_total / (loc_max * 1e-3) / 1e9, 3),
           "skew_us_per_step": round((loc_max - loc_min) * 1e3, 3),
           "exchange_us_per_step": round((headline_ms - loc_max) * 1e3, 3),
           "scaling_efficiency_vs_local": round(loc_max / headline_ms, 5) if headline_ms > 0 else None,
           "local_launch": m["launch"], "steps": K, "consistent": same and err is None}
    if wait is not None:
        out["exchange_wait_us"] = wait
    if err:
        out["error"] = err
    return out


def _exchange_wait(wl, ctx, args, fault, cap: int = 4096, allow_graph: bool = True) -> "dict | None":
    """Device-side timing of the fused exchange (XrankChannel.set_stamps): for every step of a
    short serial graph-replayed run, the finisher's wall clock at its first push and when every
    peer's partial had landed. Per rank the median / p90 of that wait (us); the rank that waits least
    arrived last (its wait is the local poll of already-landed partials), the one that waits most
    pays the skew of the local reductions plus the xGMI latency. None if unsupported."""
    ch = wl.channels[0]
    if not hasattr(ch, "set_stamps"):
        return None
    K, W = min(args.steps, cap - 8), 2
    st = torch.zeros(2 * cap, dtype=torch.int64, device=ctx.device)
    err = None
    try:
        ch.set_stamps(st.data_ptr(), cap)
        _measure(wl, wl.new_slots(W + K), ctx, args, fault, serial=True, warmup=W, site="extras",
                 allow_graph=allow_graph)
    except Exception as e:  # noqa: BLE001 - an extra must never cost the headline
        err = f"{type(e).__name__}: {e}"[:200]
    finally:
        ch.set_stamps(0, 1)
    s = st.view(-1, 2).cpu()
    s = s[s[:, 0] > 0]
    us = ((s[:, 1] - s[:, 0]).to(torch.float64) / ch.ticks_per_us).sort().values
    med = float(us[len(us) // 2]) if len(us) else float("nan")
    p90 = float(us[int(0.9 * (len(us) - 1))]) if len(us) else float("nan")
    rows = [None] * ctx.world_size
    mine = {"median": round(med, 3), "p90": round(p90, 3), "launches": int(len(us)), "error": err}
    if ctx.world_size > 1:
        torch.distributed.all_gather_object(rows, mine)
    else:
        rows = [mine]
    meds = [r["median"] for r in rows]
    return {"median_by_rank": meds, "p90_by_rank": [r["p90"] for r in rows], "min_rank_median": min(meds),
            "max_rank_median": max(meds), "launches": min(r["launches"] for r in rows),
            "errors": [r["error"] for r in rows if r["error"]] or None}


def _time_local(launch, slots: torch.Tensor, T: int, dev: torch.device) -> float:
    """Seconds this rank alone takes for T launches of ``launch`` (2 eager warm-ups; on GPUs the T
    launches are replayed from one captured graph, uploaded by an untimed replay; eager if the
    capture fails or on CPU). No collective: the candidates of every rank are timed independently
    (each GPU streams its own HBM)."""
    for i in range(2):
        launch(slots[i:i + 1])
    _sync(dev)
    sg = None
    if dev.type == "cuda":
        sg = StepGraph(lambda j: launch(slots[2 + j:3 + j]), T, dev, chunk=T, serial=True)
        if sg.capture(group_agree=False, settle_s=0.0):  # kernels only: the NCCL stream stays out
            sg.run()
            _sync(dev)
        else:
            sg = None
    t0 = time.perf_counter()
    if sg is not None:
        sg.run()
    else:
        for j in range(T):
            launch(slots[2 + j:3 + j])
    _sync(dev)
    el = time.perf_counter() - t0
    if sg is not None:
        sg.reset()
    return el


def _tune_plan(wl, ctx, args, fault, kernel, cands) -> "tuple[KernelConfig, dict]":
    """Streaming-kernel plan for this rank's shard, chosen PER RANK: every candidate is measured on
    every rank, kernel-only — the step's own local launch without the combine (a prepared launch on
    a workspace of its own, no channel: ``wl.local_launcher``), graph-replayed — in two rounds, best
    of each (a first candidate measured while the driver works on memory released just before it
    runs slow: profiles/r3_selfcheck/), and each rank keeps the plan that is fastest on ITS GPU. The
    step time of the N-GPU job is the max over ranks of (local + combine), so per-rank
    choice strictly dominates one plan for all: max_r min_p t(r, p) <= min_p max_r t(r, p).

    Failure boundary: the measurement is LOCAL (no collective, the bound
    combine untouched) and inside a try; then one bounded agreement (:func:`parallel.dist.agree`)
    of every rank's table. A candidate whose fan-in flagged an error on any rank is out for every
    rank; if any rank's tuning raised, EVERY rank keeps the tuned default (already bound) and the
    record says why; a rank that died or hangs makes the others raise PeerLost (main() prints the
    line naming the stage). Only then, with every rank's choice known, are the chosen plans bound:
    each rank re-binds its own lanes, keeping its fused channel (``wl.use_kernel`` is local — no
    collective; skipped when every rank keeps the default), and one more bounded agreement checks
    the re-binds: if one failed anywhere, every rank returns to the default plan. Fault site ``tune`` fires before the
    candidates are measured. Returns this rank's kernel config and the record (``chosen`` = rank
    0's plan, ``plan_by_rank`` = every rank's, ``gbps_by_rank`` = every rank's table)."""
    T = max(4, args.tune_steps) if args.tune_steps else _auto_tune_steps(wl.bytes_total / ctx.world_size)
    local_bytes = wl.count * wl.x.element_size()
    default_key = _plan_key(cands[0])
    res, err = {}, None
    try:
        fault.at(ctx.rank, fault.spec.step, "tune", "plan tuning")
        launchers = {}
        slots = wl.new_slots(2 + T)
        for _round in range(2):
            for c in cands:
                key = _plan_key(c)
                if res.get(key, 0.0) < 0:
                    continue
                b, u, w, win, skew = c
                if key not in launchers:
                    launchers[key] = wl.local_launcher(replace(kernel, block=b, unroll=u, wg_per_cu=w,
                                                               window=None if win < 0 else win, xcd_skew=skew))
                launch, error = launchers[key]
                el = _time_local(launch, slots, T, ctx.device)
                g = round(local_bytes * T / el / 1e9, 3)
                res[key] = -1.0 if error() != 0 else max(res.get(key, 0.0), g)
        launchers.clear()
    except Exception as e:  # noqa: BLE001 - reported through the agreement; every rank keeps the default
        err = f"{type(e).__name__}: {e}"[:200]
        print(f"[bench] rank {ctx.rank}: plan tuning failed here: {err}", file=sys.stderr, flush=True)
    forced = None
    # test hook (tests/test_xrank_gpu.py, MIREDUCE_TEST=1 only): MIREDUCE_PLAN_FOR_RANK="1=tuned default,
    # XCD skew 0;..." makes the named ranks hold another candidate, so a heterogeneous job is exercised
    # deterministically; the record marks it (forced_by_env)
    if os.environ.get("MIREDUCE_TEST") == "1":
        for item in filter(None, os.environ.get("MIREDUCE_PLAN_FOR_RANK", "").split(";")):
            r, _, key = item.partition("=")
            if r.strip() == str(ctx.rank) and any(_plan_key(c) == key for c in cands):
                forced = key
    rows = pdist.agree(ctx, "plan tuning", {"error": err, "gbps": res, "forced": forced}, _agree_timeout(args))
    rec = {"steps": T, "measure": "kernel-only local launch per rank (GB/s of the rank's shard)",
           "gbps_by_rank": [r["gbps"] for r in rows]}
    errs = [f"rank {r}: {row['error']}" for r, row in enumerate(rows) if row["error"]]
    if errs:  # every rank keeps the tuned default plan, which the workload is still bound to
        rec.update(chosen=default_key, plan_by_rank=[default_key] * ctx.world_size,
                   error="; ".join(errs)[:300], fallback="tuned default on every rank")
        return kernel, rec
    out = {k for row in rows for k, v in row["gbps"].items() if v < 0}  # a fan-in error on any rank
    picks = []
    for row in rows:
        ok = {k: v for k, v in row["gbps"].items() if k not in out}
        best = max(ok, key=ok.get) if ok else default_key
        if row["forced"] and row["forced"] not in out:
            best = row["forced"]
        picks.append(best)
    if any(row["forced"] for row in rows):
        rec["forced_by_env"] = {str(r): row["forced"] for r, row in enumerate(rows) if row["forced"]}
    mine = picks[ctx.rank]
    b, u, w, win, skew = next(c for c in cands if _plan_key(c) == mine)
    chosen = replace(kernel, block=b, unroll=u, wg_per_cu=w, window=None if win < 0 else win, xcd_skew=skew)
    if all(p == default_key for p in picks):
        rec.update(chosen=picks[0], plan_by_rank=picks)
        return kernel, rec
    bind_err = None
    try:
        wl.use_kernel(chosen, streams=1)  # local: this rank's lanes, its own plan, the same channel
    except Exception as e:  # noqa: BLE001
        bind_err = f"{type(e).__name__}: {e}"[:200]
    bad = [f"rank {r}: {row['error']}" for r, row in
           enumerate(pdist.agree(ctx, "plan binding", {"error": bind_err}, _agree_timeout(args))) if row["error"]]
    if bad:
        wl.use_kernel(kernel, streams=1)
        rec.update(chosen=default_key, plan_by_rank=[default_key] * ctx.world_size,
                   error=("binding: " + "; ".join(bad))[:300], fallback="tuned default on every rank")
        return kernel, rec
    rec.update(chosen=picks[0], plan_by_rank=picks)
    return chosen, rec


def _plans_summary(plan_by_rank: list) -> str:
    """'tuned default x6; tuned default, XCD skew -20 x2' — the per-rank plans, compactly."""
    from collections import Counter
    return "; ".join(f"{k} x{c}" if len(plan_by_rank) > 1 else k for k, c in Counter(plan_by_rank).items())


def _topology(ctx) -> dict:
    """Where the ranks ran (parallel/topology.py peer_map): hosts, physical GPUs, ranks per GPU and
    the agreed peer-access verdict of the IPC-mapped paths (collective at N > 1)."""
    from cuda_mpi_reductions_amd.parallel.topology import peer_map
    # (peer_map enters its gathers on every rank even when this rank's device query fails, so an
    # exception here is raised on every rank alike, after the collectives)
    try:
        pm = peer_map(ctx.device.index if ctx.device.index is not None else torch.cuda.current_device())
    except Exception as e:  # noqa: BLE001 - a record field must never cost the headline
        return {"error": f"{type(e).__name__}: {e}"[:200]}
    return {"hosts": len({k[0] for k in pm.keys}), "gpus": len({(k[0], k[1]) for k in pm.keys}),
            "ranks_per_gpu": pm.ranks_per_gpu,
            "peer_access": "n/a (one GPU)" if len({(k[0], k[1]) for k in pm.keys}) == 1 else
                           (pm.error or "every pair of GPUs")}


HEADLINE_RESERVE_S = 25.0  # run budget kept after the headline phase (teardown; the extras fit or are skipped)
EXTRAS_RESERVE_S = 25.0  # run budget kept after the extras (teardown, the parent's grace)
EXTRAS_MIN_S = 15.0  # an extras window shorter than this is skipped (agreed over ranks)
NONROOT_GRACE_S = 10.0  # non-root ranks' headline deadline is this much later than rank 0's
REMEASURE_MIN_S = 30.0  # headline time that must be left to re-measure over RCCL after a failed fused finish


def _budget_left(args) -> float:
    return T0 + args.budget - time.time()


def _deadline(args, requested: float, reserve: float, floor: float = 5.0) -> float:
    """A phase deadline: the requested one, cut so that ``reserve`` seconds of the run budget stay
    for what follows the phase (never below ``floor``)."""
    return max(floor, min(requested, _budget_left(args) - reserve))


_STATE: dict = {}  # what main() needs when a bounded agreement reports a lost rank (PeerLost)


def main(argv=None) -> int:
    """The bench; a rank found dead or hung by a bounded agreement (parallel.dist.PeerLost: no
    collective can complete any more) ends the job here with exactly one line from rank 0 — the
    diagnostic naming the stage during the headline phase, the verified headline (extras marked)
    after it — and status 2 (headline phase) or the headline's status."""
    try:
        return _main(argv)
    except pdist.PeerLost as e:
        rec = _STATE.get("record")
        line = rec.final(error=f"extras stopped: {e}") if rec is not None else \
            (_STATE["diag"](str(e)) if _STATE.get("diag") else None)
        if line is not None:
            _emit(line)
        import datetime
        try:  # the other ranks wait (bounded) until rank 0 has printed: an early exit of theirs would
            # make the launcher SIGTERM rank 0 first, and its line would be the generic armed one
            store = pdist._store()
            if line is not None:
                store.set("mireduce/peer-lost-line", "1")
            elif int(os.environ.get("RANK", "0")) != 0:
                store.wait(["mireduce/peer-lost-line"], datetime.timedelta(seconds=NONROOT_GRACE_S))
        except Exception:  # noqa: BLE001 - rank 0 gone too (the launcher's parent prints then)
            pass
        rc = _STATE.get("rc", 2) if _STATE.get("headline_done") else 2
        print(f"[bench] {e}: exiting with {rc}", file=sys.stderr, flush=True)
        sys.stderr.flush()
        os._exit(rc)


def _main(argv=None) -> int:
    args = parse_args(argv)
    C = native()  # fail loudly if the HIP extension is missing
    C.set_tracing(args.trace)
    if args.device != "auto":
        device_type = args.device
    else:  # CPU-rank configs (reduce.c plumbing) run on CPU ranks even on a GPU box
        device_type = "cpu" if CONFIGS[args.config].device == "cpu" else None
    fault = FaultInjector.from_flag_or_env(args.inject_fault)
    cfg = CONFIGS[args.config]
    if args.elements is not None:
        cfg = replace(cfg, n_total=args.elements)
    K, W = args.steps, args.warmup
    metric = METRIC if cfg.name == NORTH_STAR else f"reduction bandwidth (GB/s), {cfg.name}"
    # Before the process group exists the launcher's environment says who this rank is.
    rank_env, world_env = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))

    # ------------------------------------------------------------------ headline phase (deadline)
    # Armed from before the process-group rendezvous: a rank that never joins must not leave the
    # job without a line (rank 0 prints the diagnostic when the deadline passes).
    stage = {"now": "init"}
    headline_deadline = _deadline(args, args.headline_deadline, HEADLINE_RESERVE_S)

    def diag(why: "str | None" = None):
        if rank_env != 0:
            return None
        d = _no_line(world_env, (why or f"headline phase did not finish within {headline_deadline:.0f} s") +
                     f" (stage: {stage['now']}); no measurement")
        d.update(metric=metric, steps=K, warmup=W, native_source_hash=C.source_hash())
        return d

    def at_stage(name: str) -> None:
        stage["now"] = name
        _arm(diag("the process was terminated (signal) during the headline phase"))
    _STATE.update(diag=diag, record=None, headline_done=False)

    # Rank 0 owns the line, so the other ranks' deadline is a little later: on a common hang rank 0
    # reports it (stage named) rather than being torn down by a peer that gave up first.
    watch = _PhaseWatchdog("headline phase", headline_deadline + (0.0 if rank_env == 0 else NONROOT_GRACE_S), 2,
                           diag)
    headline_ends = time.time() + headline_deadline  # (rank 0's watchdog)
    # fault site "init": before this rank arms anything or joins the group (a rank that exits here
    # leaves no line of its own; one that hangs here keeps the others in the rendezvous)
    fault.at(rank_env, fault.spec.step, "init", "process-group init")
    at_stage("init")
    ctx = pdist.init(backend=None if args.backend == "auto" else args.backend, device_type=device_type,
                     timeout_s=args.pg_timeout)
    if args.gpus is None:
        args.gpus = ctx.world_size
    if args.gpus != ctx.world_size:  # (main() called directly; the __main__ launcher checks this first)
        watch.finish()
        if ctx.is_root:
            _emit(_no_line(args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={ctx.world_size}"))
        pdist.shutdown(ctx)
        return 2
    if cfg.mode == "vector":
        at_stage("vector collectives")
        rc = run_vector(args, ctx, cfg, fault)
        watch.finish()
        pdist.shutdown(ctx)
        return rc
    dev = ctx.device
    at_stage("setup")

    kernel = KernelConfig(block=args.block, unroll=args.unroll, wg_per_cu=args.wg_per_cu,
                          nontemporal=None if args.policy == "auto" else args.policy == "nt",
                          single_pass=not args.two_pass)
    collective = args.collective
    rehearse = args.rehearse_stages and dev.type == "cpu"  # the GPU-only stages in their CPU form
    fused_ok = (dev.type == "cuda" or rehearse) and not args.two_pass and cfg.op not in LOC_OPS and not args.local_only
    if collective == "fused" and not fused_ok:
        raise SystemExit("--collective fused needs GPUs, the single-pass kernel and a non-LOC operator")
    lanes = max(1, args.streams) if args.pipelined else 1
    # The cross-rank combine is issued even on one rank (--local-only skips it): N=1 runs the
    # exact step the N-GPU job runs.
    wl = scalar_workload(cfg, ctx, kernel, streams=lanes, collective="rccl" if collective == "auto" else collective,
                         always_collective=not args.local_only, xrank_timeout_s=args.xrank_timeout,
                         fault=fault).setup()
    collective_note = None
    args._headline_ends = headline_ends
    if collective == "auto":
        collective = "rccl"
        if fused_ok:
            at_stage("fused self-check")
            collective_note = _try_fused(wl, ctx, args, fault, at_stage)
            collective = "fused" if collective_note is None else "rccl"
            if collective_note and ctx.is_root:
                print(f"[bench] fused finish unavailable, using RCCL: {collective_note}", file=sys.stderr)
            if lanes > 1:
                wl.use_collective(collective, streams=lanes)

    plan_tuning = None
    explicit_plan = args.block or args.unroll or args.wg_per_cu or args.two_pass or args.policy != "auto"
    if args.collective == "auto" and collective == "fused" and lanes == 1 and not fault.on("step") \
            and (dev.type == "cuda" or rehearse) and not explicit_plan and args.plan_tune and hasattr(wl, "use_kernel"):
        es = torch.empty((), dtype=cfg.dtype).element_size()
        # (a CPU rehearsal times the large-shard candidate list over the host reducer)
        cands = _plan_candidates(1 << 40 if rehearse else wl.bytes_total / ctx.world_size, es)
        if len(cands) > 1:
            # local, kernel-only measurements, then one bounded agreement: cannot hang on a collective
            at_stage("plan tuning")
            kernel, plan_tuning = _tune_plan(wl, ctx, args, fault, kernel, cands)

    def timed(label: str) -> tuple:
        """The K timed steps, the device error words and the verification of every slot written."""
        at_stage(label)
        slots = wl.new_slots(W + K)
        m = _measure(wl, slots, ctx, args, fault, serial=not args.pipelined, warmup=W)
        err = wl.check()  # device error words (fan-in, fused finish), agreed over ranks
        seen = _ranks_seen(ctx)
        if seen != ctx.world_size:
            err = (err + "; " if err else "") + f"the process group joined {seen} ranks, not {ctx.world_size}"
        at_stage("verification")
        verified, ref = None, None
        if not args.no_verify:
            ok, ref = _verify_slots(wl, slots[:m["written"]], ctx)
            verified = ok and err is None
            if not verified and ctx.is_root:
                print(f"[bench] VERIFICATION FAILED: {ref or ''} {err or ''}", file=sys.stderr)
        elif err is not None:
            verified = False
        if err is not None and ctx.is_root:
            print(f"[bench] device error: {err}", file=sys.stderr)
        return m, err, seen, verified, ref

    m, err, seen, verified, ref = timed("timed steps")
    fused_failed = None
    if verified is False and args.collective == "auto" and collective == "fused" and ctx.world_size > 1:
        # The fused finish passed its canary and self-check but failed on the headline's own steps:
        # the number is re-measured over RCCL (same data, same plan) if the run budget has room, and
        # the sidecar keeps why. Agreed over ranks (the verdict and the budget check both are).
        why = f"fused finish failed on the headline steps ({err or 'wrong result: ' + str(ref)[:120]})"
        room = min(_budget_left(args) - HEADLINE_RESERVE_S, headline_ends - time.time()) - REMEASURE_MIN_S
        if -pdist.max_over_ranks(-float(room > 0), ctx) > 0.5:
            fused_failed = f"{why}; re-measured over RCCL"[:300]
            if ctx.is_root:
                print(f"[bench] {fused_failed}", file=sys.stderr)
            wl.use_collective("rccl", streams=lanes)
            collective, collective_note = "rccl", fused_failed
            m, err, seen, verified, ref = timed("timed steps (RCCL after the fused finish failed)")
        else:
            fused_failed = f"{why}; no time left in the headline phase to re-measure over RCCL"[:300]
            if ctx.is_root:
                print(f"[bench] {fused_failed}", file=sys.stderr)
    m_lanes = len(wl.lanes) if wl.lanes else 1
    m_issues = wl.issues_collective

    gbps = _gbps(wl, K, m["elapsed"])
    ms = m["elapsed"] / K * 1e3
    topo = _topology(ctx) if dev.type == "cuda" else None  # collective at N > 1 (cached after fused)
    record = None
    if ctx.is_root:
        world1 = ctx.world_size == 1
        if m_issues:
            combine = ("none at world 1 (a 1-rank RCCL all-reduce is issued but enqueues no kernel)" if world1 else
                       "RCCL all-reduce of the 1-element partial (torch.distributed nccl)" if ctx.backend == "nccl"
                       else f"{ctx.backend} all-reduce of the 1-element partial")
        elif collective == "fused":
            combine = ("none at world 1 (the fused finish is bound, exchanges nothing)" if world1 else
                       "fused in-kernel cross-rank finish (IPC mailboxes over xGMI, csrc/include/mireduce/xrank.hpp)")
        else:
            combine = "none (--local-only)"
        launcher = os.environ.get(LAUNCHER_ENV) or ("external" if "WORLD_SIZE" in os.environ else "single process")
        line = {  # the proof fields first: the driver keeps a bounded set of keys and a stdout tail
            "metric": metric,
            "value": round(gbps, 3),
            "unit": "GB/s",
            "n_gpus": ctx.world_size,
            "verified": verified,
            "ranks_seen": seen,
            "rccl_ranks_seen": seen if ctx.backend == "nccl" else None,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(ms, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(gbps / cfg.baseline, 3) if cfg.baseline else None,
            "dtype": "fp64" if cfg.dtype == torch.float64 else str(cfg.dtype).replace("torch.", ""),
            "data": "synthetic (on-device counter-based U[0,1) fill, untimed; random-filled array)",
            "config": {
                "model": f"{cfg.name}: {cfg.description}",
                "global_batch": wl.n_total,
                "seq_len": 1,
                "parallelism": f"dp{ctx.world_size}",
                "backend": ctx.backend,
                "n_total_elements": wl.n_total,
                "bytes_per_step": wl.bytes_total,
                "op": cfg.op.upper(),
                "collective": collective,
                "launch": m["launch"],
            },
            "launcher": launcher,
            "native_source_hash": C.source_hash(),
        }
        if args.collective == "auto" and collective != "fused" and (fused_failed or collective_note):
            # why the fused finish is not the combine: in `config`, whose values the driver's record keeps
            line["config"]["collective_reason"] = (fused_failed or collective_note)[:120]
        if plan_tuning is not None and plan_tuning.get("error"):
            # why every rank kept the tuned default plan (the tuning failed on some rank)
            line["config"]["plan_reason"] = f"plan tuning fell back to the tuned default: {plan_tuning['error']}"[:160]
        if ctx.world_size > 1 and isinstance(topo, dict) and topo.get("peer_access"):
            line["config"]["peer_access"] = str(topo["peer_access"])[:80]
        if err is not None:
            line["device_error"] = err[:300]
        detail = {
            "config_detail": {
                "collective_choice": (f"auto: {fused_failed}" if fused_failed else
                                      "auto: fused finish passed its self-check on every rank"
                                      if args.collective == "auto" and collective == "fused" else
                                      f"auto; fused unavailable: {collective_note}" if collective_note else
                                      "auto" if args.collective == "auto" else "explicit (--collective)"),
                "cross_rank_combine": combine,
                "overlap": ("serial: one stream lane, each global reduction (local reduce + combine) completes "
                            "before the next starts (reduction.cpp:319-374)") if not args.pipelined else
                           ("pipelined (step i+1 local reduce || step i all-reduce)" if m_issues
                            else f"pipelined over {m_lanes} stream lanes"),
                "streams": m_lanes,
                "kernel_plan": wl.reducer.last_plan if getattr(wl, "reducer", None) else getattr(wl, "plan", None),
                "topology": topo,
            },
            "device": dev.type,
            "per_gpu_gbps": round(gbps / ctx.world_size, 3),
            "baseline_value": cfg.baseline,
            "baseline_source": cfg.baseline_source,
            "native_ext": os.path.basename(native_path()),
            "ranks_seen_backend": ctx.backend,
            "rccl_env": _rccl_env(),
            "budget_s": args.budget,
            "headline_done_s": round(time.time() - T0, 2),
        }
        record = _Record(line, detail, args.extras_file or _default_extras_path(ctx.world_size))
        if plan_tuning is not None:
            record.extras["plan_tuning"] = plan_tuning
    rc = 0 if verified in (None, True) else 1
    if not watch.finish():
        return 2  # (unreachable: the watchdog ended the process)
    _STATE.update(record=record, rc=rc, headline_done=True)

    # ------------------------------------------------------------------ extras (watchdog; never the headline)
    # Order: the decomposition and the fused 2-lane candidate (kernels only), reduce.c's table
    # (direct collective first: no RCCL), then the RCCL step candidates, so a hang costs the fewest
    # extras; the watchdog prints the line with the summary of what has completed. Extras that no
    # longer fit in the run budget are skipped (agreed over ranks).
    room = _budget_left(args) - EXTRAS_RESERVE_S  # what the run budget leaves for the extras
    extras_deadline = max(0.01, min(args.extras_deadline, room))
    do_extras = -pdist.max_over_ranks(-float(room >= EXTRAS_MIN_S), ctx) > 0.5  # AND over ranks
    extras = record.extras if record is not None else {}
    # (skipped extras run nothing: their guard only covers writing the record)
    guard = _ExtrasWatchdog(record, extras_deadline if do_extras else 10.0, rc)

    def rearm() -> None:  # the finished headline + the extras so far, should the process be killed now
        if record is not None:
            _arm(record.final(error="the process was terminated (signal) during the extras; headline measured "
                                    "and verified before them"))
    rearm()
    if not do_extras:
        extras["skipped"] = f"run budget: {max(0.0, _budget_left(args)):.0f} s left after the headline"
    run_cands = do_extras and args.candidates and dev.type == "cuda" and hasattr(wl, "use_collective") \
        and not args.pipelined
    cap_failed = m["launch"].startswith("eager (graph capture failed")
    if do_extras and args.decompose and not args.pipelined and hasattr(wl, "local_step"):  # kernels only: first
        try:
            # (after a failed capture of the headline's collective steps another capture in this process
            # can abort it: profiles/r2_full/; the decomposition then issues its steps eagerly)
            extras["decomposition"] = _decompose(wl, ctx, args, fault, ms, allow_graph=not cap_failed)
        except Exception as e:  # noqa: BLE001 - an extra must never cost the headline
            extras["decomposition"] = {"error": f"{type(e).__name__}: {e}"[:300]}
            print(f"[bench] rank {ctx.rank}: decomposition failed: {e}", file=sys.stderr)
        rearm()
    if run_cands:  # the fused (kernel-only) candidate first: before the torch-heavy extras below
        extras["candidates"] = _candidates(wl, ctx, args, fault, collective == "fused", cap_failed, which="fused")
        rearm()
    if do_extras and args.vector_extras and dev.type == "cuda" and cfg.name == NORTH_STAR:
        extras["reduce_c_vector"] = {}
        _vector_extras(ctx, out=extras["reduce_c_vector"], progress=rearm, canary=args.canary,
                       canary_timeout=args.canary_timeout)
        rearm()
    if do_extras and args.compare_torch and dev.type == "cuda":
        extras["torch_gbps"] = round(_time_torch_reduction(wl, K, W, ctx), 3)
        rearm()
    if run_cands:  # the RCCL candidates last: a hang there costs the fewest extras
        extras.setdefault("candidates", {}).update(
            _candidates(wl, ctx, args, fault, collective == "fused", cap_failed, which="rccl"))
    if guard.finish() and record is not None:
        _emit(record.final())
    # The line is out: a teardown stuck in a collective (communicator destruction) must not hold
    # the job either, so it gets a deadline of its own and exits with the headline's status.
    teardown = _PhaseWatchdog("teardown", _deadline(args, args.teardown_deadline, 0.0), rc, lambda: None)
    fault.at(ctx.rank, fault.spec.step, site="teardown")
    _sync(dev)
    pdist.shutdown(ctx)
    teardown.finish()
    return rc


if __name__ == "__main__":
    sys.exit(main())
