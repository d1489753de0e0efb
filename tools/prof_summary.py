#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output: top kernels by time, and per-kernel PMC means.
    usage: tools/prof_summary.py <trace_dir> [<pmc_dir>]"""
import collections
import csv
import glob
import os
import sys


def main(argv):
    trace = argv[1]
    for path in glob.glob(os.path.join(trace, "*kernel_stats.csv")):
        rows = list(csv.DictReader(open(path)))
        print(f"== {path}")
        for r in rows[:10]:
            print(f"{float(r['AverageNs']) / 1e3:12.2f} us x {int(r['Calls']):5d}  {r['Name'][:110]}")
    if len(argv) > 2:
        for path in glob.glob(os.path.join(argv[2], "*counter_collection.csv")):
            agg = collections.defaultdict(list)
            for r in csv.DictReader(open(path)):
                agg[(r["Kernel_Name"][:90], r["Counter_Name"])].append(float(r["Counter_Value"]))
            print(f"== {path}")
            for (k, c), v in sorted(agg.items()):
                print(f"{c:>18} mean {sum(v) / len(v):16.1f} over {len(v):4d}  {k}")


if __name__ == "__main__":
    main(sys.argv)
