#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite (rocpd) output: per-kernel call count, total / mean / min / max
duration, and (--timeline) the gaps between consecutive dispatches.
    usage: tools/prof_db.py <results.db> [--csv out.csv] [--timeline N] [--steady SUBSTR]
--steady: for the longest back-to-back run of kernels whose name contains SUBSTR (runs split at
idle gaps > 1 ms), the period per kernel (first start to last end / count), the mean kernel
duration and how much of the run had two or more of them executing at once (multi-stream overlap).
(rocprofv3 on ROCm 7 writes <dir>/<name>_results.db unless --output-format csv is given.)"""
import argparse
import csv
import sqlite3
import statistics
import sys


def kernels(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    q = f"select {name}, start, end from kernels order by start"
    return [(n, s, e) for n, s, e in c.execute(q)]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--timeline", type=int, default=0, help="print the first N dispatches with gaps")
    ap.add_argument("--steady", default="", help="period / overlap of the longest run of matching kernels")
    a = ap.parse_args(argv)
    ks = kernels(a.db)
    by = {}
    for n, s, e in ks:
        by.setdefault(n, []).append((e - s) / 1e3)
    rows = sorted(((sum(v), n, v) for n, v in by.items()), reverse=True)
    tot = sum(r[0] for r in rows) or 1.0
    out = []
    for t, n, v in rows:
        out.append({"kernel": n, "calls": len(v), "total_us": round(t, 2), "pct": round(100 * t / tot, 2),
                    "mean_us": round(statistics.mean(v), 3), "median_us": round(statistics.median(v), 3),
                    "min_us": round(min(v), 3), "max_us": round(max(v), 3)})
    for r in out:
        print(f"{r['calls']:6d} x {r['mean_us']:10.2f} us (med {r['median_us']:9.2f}, min {r['min_us']:9.2f}) "
              f"{r['pct']:6.2f}%  {r['kernel'][:120]}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0]))
            w.writeheader()
            w.writerows(out)
    if a.timeline:
        prev = None
        for n, s, e in ks[:a.timeline]:
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"  +{gap:9.2f} us gap  {(e - s) / 1e3:9.2f} us  {n[:100]}")
            prev = e
    if a.steady:
        print(steady(ks, a.steady))
    return 0


def steady(ks, substr: str, idle_ns: float = 1e6) -> str:
    ms = sorted((s, e) for n, s, e in ks if substr in n)
    if not ms:
        return f"steady: no kernel matches {substr!r}"
    runs, cur = [], [ms[0]]
    for s, e in ms[1:]:
        if s - max(x[1] for x in cur[-4:]) > idle_ns:
            runs.append(cur)
            cur = []
        cur.append((s, e))
    runs.append(cur)
    run = max(runs, key=len)
    t0, t1 = run[0][0], max(e for _, e in run)
    busy2 = 0.0  # time with >= 2 matching kernels active (sweep over start/end events)
    ev = sorted([(s, 1) for s, _ in run] + [(e, -1) for _, e in run])
    active, last = 0, t0
    for t, d in ev:
        if active >= 2:
            busy2 += t - last
        active += d
        last = t
    n = len(run)
    dur = statistics.mean(e - s for s, e in run) / 1e3
    return (f"steady: {n} x {substr!r} back to back: period {(t1 - t0) / n / 1e3:.2f} us per kernel, "
            f"mean duration {dur:.2f} us, >= 2 running {100 * busy2 / (t1 - t0):.1f} % of the run")


if __name__ == "__main__":
    sys.exit(main())
