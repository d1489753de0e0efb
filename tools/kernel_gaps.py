#!/usr/bin/env python3
"""Per-dispatch durations and inter-kernel gaps from a rocprofv3 kernel trace.

    usage: tools/kernel_gaps.py <trace_dir> [--match reduce_stream] [--bytes 1e9]

For back-to-back dispatches of the matched kernel: median duration, median gap (end of one
dispatch to start of the next), the kernel-only bandwidth (bytes / duration) and the
step bandwidth (bytes / (duration + gap)). Answers "how much of a step is launch overhead".
"""
import argparse
import csv
import glob
import os
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="reduce_stream")
    ap.add_argument("--bytes", type=float, default=0.0)
    ap.add_argument("--skip", type=int, default=0, help="ignore the first N matched dispatches")
    a = ap.parse_args()
    rows = []
    for path in glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(path)) if re.search(a.match, r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[a.skip:]
    if len(rows) < 2:
        print("fewer than 2 matching dispatches")
        return
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    gaps = [(int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) / 1e3 for i in range(len(rows) - 1)]
    md, mg = statistics.median(dur), statistics.median(gaps)
    print(f"dispatches {len(rows)}  kernel {rows[0]['Kernel_Name'][:100]}")
    print(f"duration us: median {md:.2f} min {min(dur):.2f} max {max(dur):.2f}")
    print(f"gap us:      median {mg:.2f} min {min(gaps):.2f} max {max(gaps):.2f}")
    if a.bytes:
        print(f"kernel-only GB/s {a.bytes / md / 1e3:.1f}   step GB/s {a.bytes / (md + mg) / 1e3:.1f}")


if __name__ == "__main__":
    main()
