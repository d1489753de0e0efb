#!/usr/bin/env python3
"""Headline benchmark: reduction bandwidth (GB/s, whole node), 1B-double SUM on N MI355X.

Driver contract: ``python bench.py --gpus N --steps K --warmup W`` (N>1 under
``torch.distributed.run``, one rank per GPU, RCCL over xGMI). One *step* is one complete global
reduction of the 1e9-element float64 array (BASELINE.json config 4): every rank reduces its
contiguous 1e9/N shard with the native single-pass HIP kernel (csrc/kernels/reduce_kernels.hpp) into a
1-element slot, then the slots are all-reduced with RCCL. The array is synthetic (on-device
counter-based U[0,1) fill, untimed) and fixed in size as N grows -> strong scaling.

Timing: W untimed warm-up steps; then barrier + synchronize, K timed steps, synchronize; the
MAX elapsed time over ranks defines the measurement. Value = total bytes reduced per step x K /
elapsed / 1e9 (GB = 1e9 B, the CUDA sample's unit, reduction.cpp:744-745).

Cross-rank combine (``--collective``): ``rccl`` = a 1-element RCCL all-reduce after the local
kernel (on RCCL's stream); ``fused`` = the local kernel's last workgroup exchanges the partials
through IPC-mapped mailboxes over xGMI and folds them itself (csrc/include/mireduce/xrank.hpp),
one kernel per step. The combine is issued even at N=1 (``--local-only`` skips it), so the 1-GPU
run executes exactly the N-GPU step.

Two measurements per run: the headline ``value`` is pipelined (independent steps: step i+1's
local reduce overlaps step i's all-reduce, which runs on its own stream); ``serial_gbps`` /
``serial_ms_per_step`` time each step to completion before the next starts (the reference's
per-reduction timing, reduction.cpp:319-374). ``--serial`` makes the serial number the headline.
Both are replayed from captured hipGraphs by default (``--launch``; chunks of up to 128 steps,
captured after eager warm-up steps and replayed once untimed): eager Python issue of the RCCL
all-reduce leaves ~22 us GPU gaps per step, which at N=8 (0.14 ms per step) would cost ~15 %.
Every step's result is checked after timing against torch's own fp64 reduction of the shards
(AND over ranks).

Reference number: 92.7729 GB/s (CUDA DOUBLE SUM, mpi/CUdata.txt:2).
"""
from __future__ import annotations

import argparse
import json
from dataclasses import replace
import math
import os
import sys
import time

import torch

from cuda_mpi_reductions_amd._native import native, native_path
from cuda_mpi_reductions_amd.models import CONFIGS, LOC_OPS, NORTH_STAR, scalar_workload
from cuda_mpi_reductions_amd.ops import KernelConfig
from cuda_mpi_reductions_amd.parallel import dist as pdist
from cuda_mpi_reductions_amd.utils.fault import FaultInjector
from cuda_mpi_reductions_amd.utils.graphs import StepGraph

METRIC = "reduction bandwidth (GB/s, whole node), 1B-double sum at 1/2/4/8 MI355X"


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default=NORTH_STAR, choices=sorted(CONFIGS))
    p.add_argument("--elements", type=int, default=None, help="override the global element count")
    p.add_argument("--serial", action="store_true",
                   help="headline with no overlap between consecutive steps (default: pipelined headline, "
                        "serial reported as serial_gbps)")
    p.add_argument("--no-serial-measure", action="store_true", help="skip the second (serial) measurement")
    p.add_argument("--collective", choices=["auto", "rccl", "fused"], default="auto",
                   help="cross-rank combine: rccl = 1-element RCCL all-reduce after the local kernel; "
                        "fused = the kernel's last workgroup folds all ranks' partials via IPC mailboxes; "
                        "auto = fused if its self-check passes on every rank, else rccl (GPU scalar configs)")
    p.add_argument("--xrank-timeout", type=float, default=30.0,
                   help="fused finish: seconds a kernel waits for a peer's partial before flagging the channel")
    p.add_argument("--tune-steps", type=int, default=0,
                   help="--collective auto: steps of the short per-candidate measurement that picks the headline "
                        "combine (fused 1 lane, fused 2 lanes, RCCL pipelined); 0 = enough steps for ~30 ms of "
                        "reduction per candidate (20..400)")
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
    p.add_argument("--local-only", action="store_true",
                   help="single rank: skip the cross-rank combine (by default it is issued even at N=1)")
    p.add_argument("--streams", type=int, default=1,
                   help="alternate independent steps over this many HIP streams (each with its own workspace)")
    p.add_argument("--block", type=int, default=0)
    p.add_argument("--unroll", type=int, default=0)
    p.add_argument("--wg-per-cu", type=int, default=0)
    p.add_argument("--groups", type=int, default=0)
    p.add_argument("--policy", choices=["auto", "nt", "default"], default="auto")
    p.add_argument("--no-plan-tune", dest="plan_tune", action="store_false",
                   help="--collective auto on GPUs also measures the streaming-kernel plan for the shard "
                        "(tuned default vs the runners-up, profiles/r2_plan/); this keeps the tuned default")
    p.add_argument("--two-pass", action="store_true")
    p.add_argument("--launch", choices=["auto", "graph", "eager"], default="auto",
                   help="graph: replay the timed steps as captured hipGraphs (chunks of --graph-chunk steps); "
                        "eager: issue every step from Python; auto: graph on GPUs when capturable")
    p.add_argument("--graph-chunk", type=int, default=0,
                   help="steps per captured graph (each graph ends by joining its lanes / last all-reduce, so "
                        "fewer, longer graphs leave fewer bubbles); 0 = auto: every timed step in one graph "
                        "(<= 4096) for the in-kernel fused finish, 128 when steps issue RCCL collectives")
    p.add_argument("--inject-fault", default=None,
                   help="failure-detection test: KIND[@RANK][:STEP], KIND = exit|hang|corrupt|delay=<ms> "
                        "(steps count warm-up first; forces --launch eager)")
    p.add_argument("--pg-timeout", type=float, default=600.0, help="process-group collective timeout (s)")
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
        if fault is not None and fault.enabled and fault.at(ctx.rank, i, "bench step"):
            wl.corrupt()
        wl.collective()
    times, checks = [], []
    holder = wl.cfg.collective == "allreduce" or ctx.rank == 0
    for i in range(W, W + K):
        wl.restore()
        if fault is not None and fault.enabled and fault.at(ctx.rank, i, "bench step"):
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
    if ctx.is_root:
        print(json.dumps({
            "metric": f"MPI_Reduce-style element-wise {cfg.collective} bandwidth (GiB/s of total data, reduce.c units)",
            "value": round(gib, 3), "unit": "GiB/s", "n_gpus": ctx.world_size if dev.type == "cuda" else 0,
            "n_ranks": ctx.world_size, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": round(gib / cfg.baseline, 3) if cfg.baseline else None,
            "dtype": str(cfg.dtype).replace("torch.", ""), "device": dev.type,
            "data": "reduce.c MT19937 per-rank data" if dev.type == "cpu" else "synthetic rank-seeded device fill",
            "config": {"model": f"{cfg.name}: {cfg.description}", "global_batch": wl.count * ctx.world_size,
                       "seq_len": 1, "parallelism": f"dp{ctx.world_size}", "backend": ctx.backend,
                       "impl": wl.impl, "op": cfg.op.upper(), "count_per_rank": wl.count},
            "baseline_value": cfg.baseline, "baseline_unit": cfg.baseline_unit if cfg.baseline else None,
            "baseline_source": cfg.baseline_source or None,
            "verified": verified,
        }), flush=True)
    return 0 if verified in (None, True) else 1


REDUCE_C_OPS = ("max", "min", "sum")  # reduce.c's operations[] order = its output row order (reduce.c:26-28)


def _vector_extras(ctx, steps: int = 5) -> dict:
    """reduce.c's own measurement on this job's GPUs, next to the scalar headline. Its whole table:
    element-wise INT and DOUBLE MAX / MIN / SUM of 2 GiB of total data each (NUM_INTS / NUM_DOUBLES,
    mpi/constants.h:1-2) to root 0 (MPI_Reduce, reduce.c:76,90), over RCCL and over the direct
    one-kernel collective, plus DOUBLE SUM to every rank (all-reduce); RETRY_COUNT (5) timed
    collectives each; GiB/s of total data (reduce.c:79,93).

    ``reduce_<impl>`` / ``allreduce_<impl>``: DOUBLE SUM; ``table``: one entry per (dtype, op, impl)
    in reduce.c's row order, and ``rows``: the same as reduce.c's ``"%s %s %d %10.3lf"`` output
    lines (DATATYPE OP NODES GB/sec, reduce.c:81,95; ``impl`` selects the file in
    tools/scaling.py's results/vector_<impl>/<DT>_<OP>.txt). Errors are recorded, not raised."""
    from dataclasses import replace as _replace

    from cuda_mpi_reductions_amd.models import CONFIGS as _C, VectorReduction
    out = {"units": "GiB/s (2^30 B of total data per collective, reduce.c:93)", "dtype": "DOUBLE", "op": "SUM",
           "total_bytes": 256 * 1024 * 1024 * 8}
    # (gloo rehearsals: its GPU-tensor reduce / all_reduce is not RCCL and crashes on 1 GiB
    # tensors, so only the direct collective runs there)
    impls = ("rccl", "direct") if ctx.backend == "nccl" else ("direct",)
    table = []

    def timed(wl):
        el, ok = _time_vector(wl, ctx, steps, 1, None, True)
        return {"gibps": round(wl.bytes_total * steps / el / float(1 << 30), 3),
                "ms": round(el / steps * 1e3, 4), "verified": ok}

    for base, dt in (("xgmi_2g_int_sum_reduce", "INT"), ("xgmi_2g_double_sum_reduce", "DOUBLE")):
        for impl in impls:
            wl = None
            try:  # one registration per (dtype, impl); the operator / collective only change the launch
                wl = VectorReduction(_C[base], ctx, impl=impl, direct_timeout_s=5.0).setup()
                for op in REDUCE_C_OPS:
                    wl.cfg = _replace(_C[base], op=op)
                    r = timed(wl)
                    table.append({"dtype": dt, "op": op.upper(), "impl": impl, **r})
                    if dt == "DOUBLE" and op == "sum":
                        out[f"reduce_{impl}"] = r
                if dt == "DOUBLE":
                    wl.cfg = _replace(_C[base], collective="allreduce")
                    out[f"allreduce_{impl}"] = timed(wl)
            except Exception as e:  # noqa: BLE001 - an extra must never cost the headline
                err = {"error": f"{type(e).__name__}: {e}"[:200]}
                import traceback
                print(f"[bench] rank {ctx.rank}: reduce.c extra {dt}/{impl} failed:\n{traceback.format_exc()}",
                      file=sys.stderr)
                done = {(t["dtype"], t["op"]) for t in table if t["impl"] == impl}
                table += [{"dtype": dt, "op": op.upper(), "impl": impl, **err} for op in REDUCE_C_OPS
                          if (dt, op.upper()) not in done]
                if dt == "DOUBLE":
                    out.setdefault(f"reduce_{impl}", err)
                    out.setdefault(f"allreduce_{impl}", err)
            if wl is not None:
                wl.close()  # collective: the next registration may reuse these addresses
                del wl
            torch.cuda.empty_cache()
    out["table"] = table
    if ctx.world_size == 1:
        out["note"] = ("world 1: RCCL enqueues no work for a 1-rank in-place reduce (its GiB/s is the host "
                       "round trip only); direct is one local in -> out pass; cross-GPU numbers need N > 1")
    out["rows"] = ["%s %s %d %10.3lf" % (t["dtype"], t["op"], ctx.world_size, t["gibps"]) + f"  # {t['impl']}"
                   for t in table if "gibps" in t]
    if ctx.world_size > 1:
        out["peer_read"] = _peer_read_extra(ctx)
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
    """Streaming-kernel plans (block, unroll, workgroups per CU) worth measuring on the node for a
    shard of this size: (0, 0, 0) = the tuned default. The ranking of the top plans moves by 1-2 %
    between boxes (profiles/r2_plan/), so for the headline's 8-byte shards the bench measures the
    default against the runners-up instead of trusting one box's table."""
    if esize == 8 and bytes_per_gpu >= 3 * (1 << 30):
        return [(0, 0, 0), (512, 8, 1), (512, 16, 1)]
    if esize == 8 and bytes_per_gpu >= 768 * (1 << 20):
        return [(0, 0, 0), (256, 8, 1)]
    return [(0, 0, 0)]


def _graph_chunk(requested: int, steps: int, issues_collective: bool) -> int:
    """Steps per captured graph. Auto: one graph for all the steps when they are kernels only (the
    fused finish; measured at the 1 GB N=8 shard with 2 lanes, 1000 steps: 7.32-7.34 TB/s as one
    graph vs 7.17-7.27 in chunks of 128, profiles/r2_shard/run4.sh), 128 when every step also
    captures an RCCL collective."""
    if requested > 0:
        return requested
    return 128 if issues_collective else max(1, min(steps, 4096))


def _measure(wl, slots, ctx, args, fault, serial: bool, warmup: int, allow_graph: bool = True,
             steps: "int | None" = None) -> dict:
    """Time K steps (after ``warmup`` eager steps); returns elapsed (MAX over ranks), the launch
    mode and how many slots the timed steps wrote (graph replays rewrite the first chunk)."""
    C = native()
    dev = ctx.device
    K = args.steps if steps is None else steps

    def run(first: int, count: int):
        works = []
        wl.fork()
        for i in range(first, first + count):
            C.trace_push("bench.step")
            corrupt = fault.at(ctx.rank, i, "bench step") if fault.enabled else False
            w = wl.step(slots[i:i + 1], async_op=True, corrupt=corrupt)
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
    capturable = dev.type == "cuda" and not args.trace and not fault.enabled and \
        (not wl.issues_collective or ctx.backend == "nccl")
    if allow_graph and ((args.launch == "graph" and not fault.enabled) or (args.launch == "auto" and capturable)):
        # Capture the K timed steps as graph replays of --graph-chunk-step chunks (all ranks agree
        # on success or all fall back to eager issue); one untimed replay uploads the graphs.
        W = warmup
        sg = StepGraph(lambda j: wl.step(slots[W + j:W + j + 1], async_op=True), K, dev,
                       chunk=_graph_chunk(args.graph_chunk, K, wl.issues_collective), serial=serial,
                       fork=wl.fork, join=wl.join)
        # (kernel-only steps keep the NCCL stream out of the capture: no watchdog settle needed)
        if sg.capture(group_agree=ctx.world_size > 1, settle_s=None if wl.issues_collective else 0.0):
            launch = f"graph (chunk {sg.chunk}, {sg.reps} replays" + (f" + 1 of {sg.rem})" if sg.rem else ")")
            for g in sg.graphs:
                g.replay()
        else:
            launch = f"eager (graph capture failed: {sg.error})"
            if ctx.is_root:
                print(f"[bench] {launch}", file=sys.stderr)
            sg = None
    _sync(dev)
    pdist.barrier(ctx)
    _sync(dev)
    t0 = time.perf_counter()
    if sg is not None:
        sg.run()
    else:
        run(warmup, K)
    _sync(dev)
    t1 = time.perf_counter()
    pdist.barrier(ctx)
    elapsed = pdist.max_over_ranks(t1 - t0, ctx)
    written = warmup + (sg.chunk if sg is not None else K)
    if sg is not None:
        sg.reset()  # captured RCCL work must not outlive the communicator
    return {"elapsed": elapsed, "launch": launch, "written": written}


def _try_fused(wl, ctx) -> "str | None":
    """Switch the workload to the fused in-kernel finish and check it on every rank: 3 steps, no
    channel timeout, results equal to torch's reference. On any failure (agreed over ranks) switch
    back to RCCL and return the reason."""
    try:
        wl.use_collective("fused")  # collective; raises on every rank if any rank cannot map
    except Exception as e:  # noqa: BLE001
        wl.use_collective("rccl")
        return f"setup: {e}"[:300]
    slots = wl.new_slots(3)
    for i in range(3):
        wl.step(slots[i:i + 1])
    _sync(ctx.device)
    err = wl.check()
    if err is None:
        ok, ref = _verify_slots(wl, slots, ctx)
        if not ok:
            err = f"self-check mismatch: {ref}"
    if err is not None:
        wl.use_collective("rccl")
    return err


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


class _ExtrasWatchdog:
    """Deadline for the reduce.c extras. If it passes first, rank 0 prints the finished headline
    line (``reduce_c_vector`` = the timeout) and every rank exits with the headline's status: a
    hung extra (e.g. one rank failing inside a collective while the others wait in it) must not
    hold the run until the process-group timeout and lose the measured metric."""

    def __init__(self, line: "dict | None", deadline_s: float, rc: int):
        import threading
        self._line, self._deadline, self._rc = line, deadline_s, rc
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
            if self._line is not None:
                line = dict(self._line)
                line["reduce_c_vector"] = {"error": f"extras did not finish within {self._deadline:.0f} s "
                                                    "(headline measured and verified before them)"}
                print(json.dumps(line), flush=True)
            print(f"[bench] reduce.c extras exceeded {self._deadline:.0f} s: exiting with the headline",
                  file=sys.stderr, flush=True)
            os._exit(self._rc)

    def finish(self) -> bool:
        """True if the extras finished before the deadline (the caller prints the line)."""
        with self._lock:
            self._timer.cancel()
            if self._done:
                return False
            self._done = True
            return True


def main(argv=None) -> int:
    args = parse_args(argv)
    C = native()  # fail loudly if the HIP extension is missing
    C.set_tracing(args.trace)
    if args.device != "auto":
        device_type = args.device
    else:  # CPU-rank configs (reduce.c plumbing) run on CPU ranks even on a GPU box
        device_type = "cpu" if CONFIGS[args.config].device == "cpu" else None
    fault = FaultInjector.from_flag_or_env(args.inject_fault)
    ctx = pdist.init(backend=None if args.backend == "auto" else args.backend, device_type=device_type,
                     timeout_s=args.pg_timeout)
    if args.gpus != ctx.world_size and ctx.is_root:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={ctx.world_size}; using {ctx.world_size}",
              file=sys.stderr)
    cfg = CONFIGS[args.config]
    if args.elements is not None:
        cfg = replace(cfg, n_total=args.elements)
    if cfg.mode == "vector":
        rc = run_vector(args, ctx, cfg, fault)
        pdist.shutdown(ctx)
        return rc
    kernel = KernelConfig(block=args.block, unroll=args.unroll, wg_per_cu=args.wg_per_cu,
                          groups=args.groups,
                          nontemporal=None if args.policy == "auto" else args.policy == "nt",
                          single_pass=not args.two_pass)
    collective = args.collective
    fused_ok = ctx.device.type == "cuda" and not args.two_pass and cfg.op not in LOC_OPS and not args.local_only
    if collective == "fused" and not fused_ok:
        raise SystemExit("--collective fused needs GPUs, the single-pass kernel and a non-LOC operator")
    # The cross-rank combine is issued even on one rank (--local-only skips it): N=1 runs the
    # exact step the N-GPU job runs.
    wl = scalar_workload(cfg, ctx, kernel, streams=args.streams, collective="rccl" if collective == "auto" else collective,
                         always_collective=not args.local_only, xrank_timeout_s=args.xrank_timeout).setup()
    collective_note = None
    if collective == "auto":
        collective = "rccl"
        if fused_ok:
            collective_note = _try_fused(wl, ctx)
            collective = "fused" if collective_note is None else "rccl"
            if collective_note and ctx.is_root:
                print(f"[bench] fused finish unavailable, using RCCL: {collective_note}", file=sys.stderr)
    K, W = args.steps, args.warmup
    dev = ctx.device

    primary_serial = args.serial
    tuning, tune_steps = None, 0
    plan_tuning = None
    explicit_plan = args.block or args.unroll or args.wg_per_cu or args.two_pass or args.policy != "auto"
    if args.collective == "auto" and not primary_serial and not fault.enabled and dev.type == "cuda" \
            and not explicit_plan and args.plan_tune and hasattr(wl, "use_kernel"):
        cands = _plan_candidates(wl.bytes_total / ctx.world_size, torch.empty((), dtype=cfg.dtype).element_size())
        if len(cands) > 1:
            # Same protocol as the combine tuning below (graph replay, MAX over ranks, two rounds,
            # best of each), one lane, with the combine the self-check settled on.
            T = max(4, args.tune_steps) if args.tune_steps else _auto_tune_steps(wl.bytes_total / ctx.world_size)
            plan_tuning = {}
            for _round in range(2):
                for b, u, w in cands:
                    key = "tuned default" if b == 0 else f"{b}x{u}x{w}"
                    wl.use_kernel(replace(kernel, block=b, unroll=u, wg_per_cu=w), streams=1)
                    mt = _measure(wl, wl.new_slots(2 + T), ctx, args, fault, serial=False, warmup=2, steps=T)
                    g = round(wl.bytes_total * T / mt["elapsed"] / 1e9, 3)
                    if wl.check() is not None:  # a timed-out fused exchange: discard the point
                        g = -1.0
                    plan_tuning[key] = g if g < 0 else max(plan_tuning.get(key, 0.0), g)
            best = max(plan_tuning, key=plan_tuning.get)
            b, u, w = next(c for c in cands if ("tuned default" if c[0] == 0 else f"{c[0]}x{c[1]}x{c[2]}") == best)
            kernel = replace(kernel, block=b, unroll=u, wg_per_cu=w)
            wl.use_kernel(kernel, streams=args.streams)
    if args.collective == "auto" and collective == "fused" and not primary_serial and not fault.enabled:
        # Pick the headline combine by a short measurement of each candidate (same graph-replay
        # protocol, MAX over ranks, so every rank picks the same): the in-kernel fused finish on one
        # stream lane or two, or the RCCL all-reduce overlapped with the next local reduce.
        # Two rounds, best of each candidate: the first candidate of round 1 otherwise pays for
        # the GPU ramping its clocks (measured: -2 % at 8 GB on an otherwise equal kernel).
        T = max(4, args.tune_steps) if args.tune_steps else _auto_tune_steps(wl.bytes_total / ctx.world_size)
        tuning, tune_steps = {}, T
        for _round in range(2):
            for coll, nl in (("fused", 1), ("fused", 2), ("rccl", 1)):
                key = f"{coll}_{nl}lane"
                if tuning.get(key, 0.0) < 0:
                    continue  # failed in round 1
                wl.use_collective(coll, streams=nl)
                mt = _measure(wl, wl.new_slots(2 + T), ctx, args, fault, serial=False, warmup=2, steps=T)
                g = round(wl.bytes_total * T / mt["elapsed"] / 1e9, 3)
                if coll == "fused" and wl.check() is not None:  # a timed-out exchange: never pick it
                    g = -1.0
                tuning[key] = g if g < 0 else max(tuning.get(key, 0.0), g)
        best = max(tuning, key=tuning.get)
        collective, nl = best.split("_")[0], int(best.split("_")[1][0])
        wl.use_collective(collective, streams=nl)
    slots = wl.new_slots(W + K)
    m1 = _measure(wl, slots, ctx, args, fault, serial=primary_serial, warmup=W)
    m1_lanes = len(wl.lanes) if wl.lanes else 1
    m1_issues = wl.issues_collective
    m1_err = wl.check()  # before any re-bind below drops the headline's channels
    m2, serial_runs = None, {}
    if not primary_serial and not wl.issues_collective and len(wl.lanes) <= 1:
        m2 = m1  # one kernel per step (fused finish): the pipelined run IS the serial run
    elif not primary_serial and not args.no_serial_measure:
        # The honest per-reduction number: every step completes (local reduce AND cross-rank
        # combine) before the next one starts (reduction.cpp:319-374 times each reduction to
        # completion), on one stream lane. Reported next to the pipelined headline, with the
        # faster combine for that protocol: when the fused finish passed its self-check both it
        # (one kernel per step) and the RCCL all-reduce are measured, else the headline's combine.
        # (Every slot is verified after all measurements — the torch reference pass between two
        # timed runs cost the following one ~6 % — while a candidate's channel errors are read
        # before the next re-bind drops its channels.)
        fused_ok_here = tuning is not None and tuning.get("fused_1lane", -1.0) > 0
        for c in (["fused", "rccl"] if fused_ok_here else [wl.collective]):
            if len(wl.lanes) > 1 or c != wl.collective:
                wl.use_collective(c, streams=1)
            s2 = wl.new_slots(min(W, 2) + K)
            # a capture that already failed (e.g. gloo collectives on GPU tensors) is not retried
            m = _measure(wl, s2, ctx, args, fault, serial=True, warmup=min(W, 2),
                         allow_graph=not m1["launch"].startswith("eager (graph capture failed"))
            m["collective"], m["slots"] = c, s2
            m["err"] = wl.check()  # before the next re-bind drops this candidate's channels
            serial_runs[c] = m
        m2 = min(serial_runs.values(), key=lambda m: m["elapsed"])

    verified = None
    err = m1_err or next((m["err"] for m in serial_runs.values() if m["err"]), None)
    if not args.no_verify:
        ok, ref = _verify_slots(wl, slots[:m1["written"]], ctx)
        for m in serial_runs.values():
            ok = _verify_slots(wl, m["slots"][:m["written"]], ctx)[0] and ok
        verified = ok and err is None
        if not verified and ctx.is_root:
            print(f"[bench] VERIFICATION FAILED: {ref or ''} {err or ''}", file=sys.stderr)
    elif err is not None:
        verified = False

    torch_gbps = None
    if args.compare_torch and dev.type == "cuda":
        torch_gbps = _time_torch_reduction(wl, K, W, ctx)
    bytes_step = wl.bytes_total
    elapsed = m1["elapsed"]
    gbps = bytes_step * K / elapsed / 1e9
    ms = elapsed / K * 1e3
    lanes = m1_lanes
    line = None
    if ctx.is_root:
        if m1_issues:
            combine = "RCCL all-reduce of the 1-element partial (torch.distributed nccl)" \
                if ctx.backend == "nccl" else f"{ctx.backend} all-reduce of the 1-element partial"
        elif collective == "fused":
            combine = "fused in-kernel cross-rank finish (IPC mailboxes over xGMI, csrc/include/mireduce/xrank.hpp)"
        else:
            combine = "none (--local-only)"
        line = {
            "metric": METRIC if cfg.name == NORTH_STAR else f"reduction bandwidth (GB/s), {cfg.name}",
            "value": round(gbps, 3),
            "unit": "GB/s",
            "n_gpus": ctx.world_size,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(ms, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(gbps / cfg.baseline, 3) if cfg.baseline else None,
            "dtype": "fp64" if cfg.dtype == torch.float64 else str(cfg.dtype).replace("torch.", ""),
            "device": dev.type,
            "data": "synthetic (on-device counter-based U[0,1) fill, untimed; random-filled array)",
            "config": {
                "model": f"{cfg.name}: {cfg.description}",
                "global_batch": wl.n_total,
                "seq_len": 1,
                "parallelism": f"dp{ctx.world_size}",
                "backend": ctx.backend,
                "n_total_elements": wl.n_total,
                "bytes_per_step": bytes_step,
                "op": cfg.op.upper(),
                "collective": collective + (f" (auto; fused unavailable: {collective_note})" if collective_note else
                                            " (auto-tuned)" if tuning is not None else
                                            " (auto)" if args.collective == "auto" else ""),
                "cross_rank_combine": combine,
                "overlap": "serial (each step completes before the next)" if primary_serial else
                           ("pipelined (step i+1 local reduce || step i all-reduce)" if m1_issues
                            else f"pipelined over {lanes} stream lanes" if lanes > 1 else
                            "serial (one kernel per step: reduce + in-kernel combine)"),
                "streams": lanes,
                "launch": m1["launch"],
                "kernel_plan": wl.reducer.last_plan if getattr(wl, "reducer", None) else getattr(wl, "plan", None),
            },
            "per_gpu_gbps": round(gbps / ctx.world_size, 3),
            "baseline_value": cfg.baseline,
            "baseline_source": cfg.baseline_source,
            "verified": verified,
            "native_ext": os.path.basename(native_path()),
        }
        if tuning is not None:
            line["collective_tuning"] = {"steps": tune_steps, "gbps": tuning,
                                         "chosen": f"{collective}_{lanes}lane"}
        if plan_tuning is not None:
            line["plan_tuning"] = {"gbps": plan_tuning, "chosen": max(plan_tuning, key=plan_tuning.get)}
        if m2 is not None:
            line["serial_gbps"] = round(bytes_step * K / m2["elapsed"] / 1e9, 3)
            line["serial_ms_per_step"] = round(m2["elapsed"] / K * 1e3, 5)
            line["serial_launch"] = m2["launch"]
            line["serial_collective"] = m2.get("collective", collective)
            if len(serial_runs) > 1:
                line["serial_candidates_gbps"] = {c: round(bytes_step * K / m["elapsed"] / 1e9, 3)
                                                  for c, m in serial_runs.items()}
        if torch_gbps is not None:
            line["torch_gbps"] = round(torch_gbps, 3)  # same data, torch's own reduction kernels
    rc = 0 if verified in (None, True) else 1
    if args.vector_extras and dev.type == "cuda" and cfg.name == NORTH_STAR:
        # The extras run after the headline is final; a watchdog prints the headline (extras marked
        # as timed out) and ends the process if they hang, so they can never cost the metric.
        guard = _ExtrasWatchdog(line, args.extras_deadline, rc)
        extras = _vector_extras(ctx)
        if guard.finish() and line is not None:
            line["reduce_c_vector"] = extras
            print(json.dumps(line), flush=True)
    elif line is not None:
        print(json.dumps(line), flush=True)
    _sync(dev)
    pdist.shutdown(ctx)
    return rc


if __name__ == "__main__":
    sys.exit(main())
