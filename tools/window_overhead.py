#!/usr/bin/env python3
"""Where the fixed cost of bench.py's timed window goes (round 5: at the N=8 shard, 1 GB per GPU,
ms_per_step was 140.2 us at K=20 and 137.7 us at K=200, i.e. ~55 us per window, ~2 % of a K=20
window, `profiles/r5_window/`).

The timed window is bench.py's: synchronize, t0, replay one captured graph of K dependent bound
launches, synchronize, t1. Here each window also records a hipEvent just before and just after the
replay, and the host time at which the replay call returned, so the window splits into

* ``enqueue``  t0 -> the replay call returned (host);
* ``gpu``      the two events' elapsed time (first packet to last kernel, device clock);
* ``rest``     host total - gpu: launch-to-first-kernel latency plus the synchronize's wake-up.

Variants (interleaved rounds): ``plain`` (as bench.py), ``warm`` (a tiny kernel enqueued and
synchronised just before t0, in case the GPU idles down between windows), ``spin`` (poll the end
event with ``query()`` instead of a blocking synchronize), ``eager`` (the K bound launches issued
one by one, no graph) and ``split`` (a one-step graph, then a (K-1)-step one: the GPU can start
while the longer graph is still being submitted), ``barrier`` (bench.py's bracket: an RCCL
barrier of a 1-rank process group, then synchronize) and ``barrier_settle`` (the same, then 0.25 s
for ProcessGroupNCCL's watchdog to retire the barrier's work before t0); ``bench`` (bench.py's
sequence: the untimed replay of the same graph, synchronize, barrier, synchronize, t0) and
``bench_nosync`` (the same without the first synchronize: the barrier queues behind the replay).

    python tools/window_overhead.py --elements 125000000 --steps 20,200 --rounds 5
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cuda_mpi_reductions_amd.ops import Reducer, fill_  # noqa: E402
from cuda_mpi_reductions_amd.utils.graphs import StepGraph  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--elements", type=float, default=125e6)
    ap.add_argument("--steps", default="20,200")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    ap.add_argument("--variants", default="plain,warm,spin,eager,split,barrier,barrier_settle")
    ap.add_argument("--fused", action="store_true", help="bind the fused cross-rank finish (a 1-rank channel), "
                    "as bench.py's headline step does")
    a = ap.parse_args(argv)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    variants = a.variants.split(",")
    if any(v.startswith(("barrier", "bench")) for v in variants):  # bench.py's bracket: an RCCL barrier first
        from cuda_mpi_reductions_amd.parallel import dist as pdist
        ctx = pdist.init()
    n = int(a.elements)
    x = torch.empty(n, dtype=torch.float64, device=dev)
    fill_(x, "uniform", seed=3)
    red = Reducer(dev)
    slots = torch.zeros(1024, dtype=torch.float64, device=dev)
    ch = None
    if a.fused:
        from cuda_mpi_reductions_amd.parallel.xrank import open_channel
        ch = open_channel(dev)
    b = red.bind(x, "sum", torch.float64, out=slots[:1], xrank=ch)
    stream = torch.cuda.current_stream(dev)
    ks = [int(k) for k in a.steps.split(",")]
    def step(j):
        b.launch(torch.cuda.current_stream(dev).cuda_stream, slots[j % 1024:j % 1024 + 1].data_ptr())

    graphs, heads, tails = {}, {}, {}
    for k in ks:
        for store, n_steps, first in ((graphs, k, 0), (heads, 1, 0), (tails, k - 1, 1)):
            sg = StepGraph(lambda j, f=first: step(f + j), n_steps, dev, chunk=n_steps, serial=True)
            assert sg.capture(), sg.error
            sg.run()
            store[k] = sg
    torch.cuda.synchronize(dev)
    tiny = torch.zeros(1, device=dev)
    res = {}
    for _ in range(a.rounds):
        for k in ks:
            for how in variants:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if how == "warm":
                    tiny.add_(1)
                if how.startswith("bench"):  # bench.py: the untimed replay of the same graph first
                    graphs[k].run()
                    if how == "bench":
                        torch.cuda.synchronize(dev)
                    pdist.barrier(ctx)  # (bench_nosync: the barrier queues behind the replay)
                torch.cuda.synchronize(dev)
                if how.startswith("barrier"):
                    pdist.barrier(ctx)
                    torch.cuda.synchronize(dev)
                    if how == "barrier_settle":  # let ProcessGroupNCCL's watchdog retire the barrier's work
                        time.sleep(0.25)
                t0 = time.perf_counter()
                e0.record(stream)
                if how == "eager":  # K bound launches issued one by one (no graph)
                    for j in range(k):
                        step(j)
                elif how == "split":  # a 1-step graph first, so the GPU starts while the rest is enqueued
                    heads[k].run()
                    tails[k].run()
                else:
                    graphs[k].run()
                e1.record(stream)
                t_enq = time.perf_counter()
                if how == "spin":
                    while not e1.query():
                        pass
                else:
                    torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                gpu = e0.elapsed_time(e1) * 1e-3
                host = t1 - t0
                res.setdefault((k, how), []).append({"host_us": host * 1e6, "enqueue_us": (t_enq - t0) * 1e6,
                                                     "gpu_us": gpu * 1e6, "rest_us": (host - gpu) * 1e6})
    print("| K | variant | host us/step | gpu us/step | window: enqueue us | window: host - gpu us |")
    print("|---|---|---|---|---|---|")
    rows = []
    for (k, how), vs in res.items():
        med = {f: statistics.median(v[f] for v in vs) for f in vs[0]}
        print(f"| {k} | {how} | {med['host_us'] / k:.2f} | {med['gpu_us'] / k:.2f} | {med['enqueue_us']:.1f} | "
              f"{med['rest_us']:.1f} |")
        rows.append({"k": k, "variant": how, **{f: round(v, 2) for f, v in med.items()}})
    ok = abs(float(slots[0].item()) - float(x.sum().item())) <= 1e-9 * abs(float(x.sum().item()))
    print(f"verified {ok}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"elements": n, "rows": rows, "verified": ok}, f, indent=1)
    for store in (graphs, heads, tails):
        for sg in store.values():
            sg.reset()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
