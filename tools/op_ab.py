#!/usr/bin/env python3
"""Same-box A/B of the streaming reduction across (dtype, op) pairs and plan variants, in
interleaved rounds (every variant of every pair timed once per round, so box drift hits all alike).
Written for BASELINE config 3 (256M int64 MIN), which ran ~1 % below the same-size double SUM in
round 5 (`profiles/r5_configs/`): is the gap the operator's instructions or the plan?

Each sample is ``--reps`` back-to-back launches between two events (the reduction app's
``--batch-timing`` shape); GB/s = bytes read / time, GB = 1e9 B. Results are checked against a
torch reference of the same array.

    python tools/op_ab.py --n 268435456 --pairs float64:sum,int64:min,int64:sum \\
        --variants "auto;xcd_skew=0;window=2" --rounds 5
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cuda_mpi_reductions_amd._native import native  # noqa: E402
from cuda_mpi_reductions_amd.ops import Reducer, default_acc_dtype, dtype_code, fill_, op_code  # noqa: E402

KNOBS = ("block", "unroll", "window", "xcd_skew", "policy", "wg_per_cu")


def parse_variants(text: str) -> list:
    """"auto;xcd_skew=0;window=2,unroll=4" -> [("auto", {}), ("xcd_skew=0", {...}), ...]."""
    out = []
    for v in (t.strip() for t in text.split(";")):
        if not v:
            continue
        kw = {}
        if v != "auto":
            for item in v.split(","):
                k, _, val = item.partition("=")
                if k not in KNOBS:
                    raise SystemExit(f"unknown knob {k!r} (one of {', '.join(KNOBS)})")
                kw[k] = int(val)
        out.append((v, kw))
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--n", type=float, default=float(1 << 28))
    ap.add_argument("--pairs", default="float64:sum,int64:min,int64:max,int64:sum,float64:min")
    ap.add_argument("--variants", default="auto;xcd_skew=0;xcd_skew=20")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    C = native()
    dev = torch.device("cuda", 0)
    n = int(a.n)
    s = torch.cuda.current_stream(dev).cuda_stream
    red = Reducer(dev)
    variants = parse_variants(a.variants)
    pairs = []
    for item in a.pairs.split(","):
        dt_name, op = item.split(":")
        dt = getattr(torch, dt_name)
        x = torch.empty(n, dtype=dt, device=dev)
        fill_(x, "uniform", seed=11)
        acc = default_acc_dtype(dt, op)
        ref = {"sum": lambda t: t.to(torch.float64 if dt.is_floating_point else torch.int64).sum(),
               "min": lambda t: t.min(), "max": lambda t: t.max()}[op](x).item()
        pairs.append((item, x, op, acc, ref))
    res, plans = {}, {}
    for r in range(a.rounds):
        for item, x, op, acc, ref in pairs:
            o = torch.zeros(1, dtype=acc, device=dev)
            for name, kw in variants:
                def go():
                    return C.reduce(red.ws, x.data_ptr(), n, dtype_code(x.dtype), op_code(op), dtype_code(acc),
                                    o.data_ptr(), s, **kw)
                plans[(item, name)] = go()  # warm
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    go()
                e1.record()
                torch.cuda.synchronize(dev)
                t = e0.elapsed_time(e1) * 1e-3 / a.reps
                got = o.item()
                tol = 1e-9 * abs(ref) + 1e-6 if x.dtype.is_floating_point and op == "sum" else 0
                ok = abs(got - ref) <= tol
                res.setdefault((item, name), []).append((x.numel() * x.element_size() / t / 1e9, ok))
    print("| pair | variant | plan | GB/s per round | median | verified |")
    print("|---|---|---|---|---|---|")
    rows = []
    for (item, name), vs in res.items():
        p = plans[(item, name)]
        plan = f"{p.get('block')}x{p.get('unroll')} grid {p.get('grid')} win {p.get('window')} skew {p.get('xskew')}"
        med = statistics.median(v for v, _ in vs)
        ok = all(k for _, k in vs)
        print(f"| {item} | {name} | {plan} | {' '.join('%.1f' % v for v, _ in vs)} | {med:.1f} | {ok} |")
        rows.append({"pair": item, "variant": name, "plan": p, "gbps": [round(v, 1) for v, _ in vs],
                     "median": round(med, 1), "verified": ok})
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"n": n, "reps": a.reps, "rounds": a.rounds, "rows": rows}, f, indent=1)
    return 0 if all(r["verified"] for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
