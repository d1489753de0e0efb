#!/usr/bin/env python3
"""Per-kernel duration statistics of the streaming reduction in rocprofv3 databases, counting only
dispatches that ran alone (no other kernel overlapping them: multi-lane candidates overlap two
reductions, which stretches both). For same-box A/B runs (profiles/r3_regress/).
    usage: tools/ab_kernels.py <results.db> [...]   (one table row per db and kernel variant)"""
import sqlite3
import statistics
import sys


def solo_durations(db, needle="reduce_stream"):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = sorted(c.execute(f"select {name}, start, end from kernels"), key=lambda r: r[1])
    out = {}
    for i, (n, s, e) in enumerate(rows):
        if needle not in n:
            continue
        lo = rows[i - 1][2] if i else -1
        hi = rows[i + 1][1] if i + 1 < len(rows) else float("inf")
        if lo > s or hi < e:  # overlapped by the previous or the next dispatch
            continue
        out.setdefault(n, []).append((e - s) / 1e3)
    return out


def short(n):
    return n.split("reduce_stream<")[-1].split(">(")[0] if "reduce_stream<" in n else n[:60]


def main(argv):
    print("| db | kernel | solo dispatches | median us | mean us | min us |")
    print("|---|---|---|---|---|---|")
    for db in argv:
        for n, d in sorted(solo_durations(db).items(), key=lambda kv: -len(kv[1])):
            if len(d) < 3:
                continue
            print(f"| {db} | {short(n)} | {len(d)} | {statistics.median(d):.1f} | {statistics.mean(d):.1f} | {min(d):.1f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
