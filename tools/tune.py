#!/usr/bin/env python3
"""Kernel-parameter sweep for the streaming reduction kernel, in ONE process with interleaved
rounds (cdna_hip_programming.md §5.4 rule 24: variants x rounds, report median and min).

    python tools/tune.py --dtype float64 --op sum --n 1e9 --rounds 5 --iters 20 [--json out.json]

Each variant is timed with hipEvents over `iters` back-to-back launches; variants are visited in
a fresh order every round so clock/thermal drift spreads over all of them.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import random
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cuda_mpi_reductions_amd.ops import KernelConfig, Reducer, fill_  # noqa: E402

DT = {"int32": torch.int32, "int64": torch.int64, "float32": torch.float32, "float64": torch.float64,
      "bfloat16": torch.bfloat16, "float16": torch.float16}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--dtype", default="float64", choices=sorted(DT))
    p.add_argument("--op", default="sum")
    p.add_argument("--n", type=float, default=1e9)
    p.add_argument("--ns", default="", help="comma list of sizes (overrides --n); one sweep per size")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--blocks", default="256,512")
    p.add_argument("--unrolls", default="2,4,8")
    p.add_argument("--wgs", default="0,2,4,8")
    p.add_argument("--policies", default="nt,default")
    p.add_argument("--windows", default="0", help="comma list of explicit load windows (0 = hipcc's schedule, 2, 4; "
                                                  "non-nt / unsupported plans fall back to 0 and are skipped)")
    p.add_argument("--json", default="")
    p.add_argument("--top", type=int, default=12)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    sizes = [int(float(v)) for v in a.ns.split(",")] if a.ns else [int(a.n)]
    dt = DT[a.dtype]
    xall = torch.empty(max(sizes), dtype=dt, device=dev)
    fill_(xall, "uniform" if dt.is_floating_point else "fullrange")
    results = []
    for n in sizes:
        results.append(sweep(a, xall[:n], n, dt, dev))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"dtype": a.dtype, "op": a.op, "sweeps": results}, f, indent=1)


def sweep(a, x, n, dt, dev):
    es = x.element_size()
    variants = []
    for b, u, w, pol, win in itertools.product(
        [int(v) for v in a.blocks.split(",")], [int(v) for v in a.unrolls.split(",")],
        [int(v) for v in a.wgs.split(",")], a.policies.split(","), [int(v) for v in a.windows.split(",")]):
        if win and (pol == "default" or b not in (256, 512) or u > 8 or u % win):
            continue  # no such window variant (reduce_kernels.hpp window_ok)
        variants.append(KernelConfig(block=b, unroll=u, wg_per_cu=w,
                                     nontemporal=None if pol == "auto" else pol == "nt", window=win))
    r = Reducer(dev)
    from cuda_mpi_reductions_amd.ops import default_acc_dtype
    out = torch.empty(1, dtype=default_acc_dtype(dt, a.op), device=dev)
    times = {i: [] for i in range(len(variants))}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ref = None
    for rnd in range(a.rounds):
        order = list(range(len(variants)))
        random.Random(rnd).shuffle(order)
        for i in order:
            cfg = variants[i]
            r(x, a.op, out.dtype, out=out, config=cfg)  # warm
            e0.record()
            for _ in range(a.iters):
                r(x, a.op, out.dtype, out=out, config=cfg)
            e1.record()
            e1.synchronize()
            times[i].append(e0.elapsed_time(e1) / a.iters)
            v = out.item()
            if ref is None:
                ref = v
            elif dt.is_floating_point and a.op == "sum":
                assert abs(v - ref) <= (1e-9 if out.dtype == torch.float64 else 1e-5) * abs(ref), (cfg, v, ref)
            else:
                assert v == ref, (cfg, v, ref)
        print(f"[tune] round {rnd + 1}/{a.rounds} done", flush=True)
    rows = []
    for i, cfg in enumerate(variants):
        med = statistics.median(times[i])
        mn = min(times[i])
        rows.append({
            "block": cfg.block, "unroll": cfg.unroll, "wg_per_cu": cfg.wg_per_cu,
            "policy": {None: "auto", True: "nt", False: "default"}[cfg.nontemporal],
            "window": cfg.window,
            "median_ms": med, "min_ms": mn,
            "median_TBps": n * es / (med * 1e-3) / 1e12, "best_TBps": n * es / (mn * 1e-3) / 1e12,
        })
    rows.sort(key=lambda r_: r_["median_ms"])
    print(f"dtype={a.dtype} op={a.op} n={n} bytes={n * es} rounds={a.rounds} iters={a.iters}")
    top = a.top if a.top > 0 else len(rows)
    print(f"{'block':>5} {'unroll':>6} {'wg/cu':>5} {'policy':>7} {'win':>3} {'median ms':>10} {'TB/s med':>9} {'TB/s best':>9}")
    for row in rows[:top]:
        print(f"{row['block']:>5} {row['unroll']:>6} {row['wg_per_cu']:>5} {row['policy']:>7} {row['window']:>3} "
              f"{row['median_ms']:>10.4f} {row['median_TBps']:>9.3f} {row['best_TBps']:>9.3f}")
    return {"n": n, "bytes": n * es, "rows": rows}


if __name__ == "__main__":
    main()
