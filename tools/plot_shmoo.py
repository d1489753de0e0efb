#!/usr/bin/env python3
"""Plot `reduction --shmoo` CSV output (n,bytes,kernel,avg_ms,GB/s): bandwidth vs array size, one
line per kernel (0..6 Harris ladder, 7 mireduce single-pass, 8 two-launch).
    python tools/plot_shmoo.py profiles/r1_bench/shmoo_double_sum.csv -o profiles/r1_bench/shmoo_double_sum.png
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("-o", "--out", default="shmoo.png")
    ap.add_argument("--title", default="MI355X reduction shmoo (float64 SUM)")
    a = ap.parse_args()
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    series = collections.defaultdict(list)
    with open(a.csv) as f:
        lines = f.read().splitlines()
        start = next(i for i, ln in enumerate(lines) if ln.startswith("n,bytes,kernel"))
        for row in csv.DictReader(lines[start:]):
            series[int(row["kernel"])].append((int(row["bytes"]), float(row["GB/s"])))
    names = {0: "k0 interleaved/divergent", 1: "k1 interleaved/strided", 2: "k2 sequential", 3: "k3 add-on-load",
             4: "k4 last wave unrolled", 5: "k5 fully unrolled", 6: "k6 = reference kernel 6 (64 blocks)",
             7: "k7 mireduce single-pass", 8: "k8 mireduce two-launch"}
    fig, ax = plt.subplots(figsize=(7.5, 5))
    for k in sorted(series):
        pts = sorted(series[k])
        ax.plot([p[0] for p in pts], [p[1] for p in pts], "-o", ms=3, lw=2 if k >= 7 else 1, label=names.get(k, k))
    ax.axhline(92.7729, ls="--", color="gray", label="reference CUDA DOUBLE SUM (92.77 GB/s)")
    ax.set_xscale("log", base=2)
    ax.set_yscale("log")
    ax.set_xlabel("array bytes")
    ax.set_ylabel("GB/s (1e9 B)")
    ax.set_title(a.title)
    ax.legend(fontsize=7, loc="upper left")
    fig.tight_layout()
    fig.savefig(a.out, dpi=120)
    print(a.out)


if __name__ == "__main__":
    main()
