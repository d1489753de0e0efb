#!/usr/bin/env python3
"""Plots in the style of the reference's mpi/makePlots.gp:1-40: bandwidth vs rank count per op,
one figure per dtype, single-GPU results as horizontal reference lines. gnuplot is not installed
in this image, so this uses matplotlib (tools/makePlots.gp is the gnuplot twin).

    python tools/plot.py --results results/ --out plots/ [--reference-cuda] [--single INT:SUM=7200,...]
        [--label "8-CPU MPICH" --xlabel "MPI ranks (CPU cores)"]
"""
import argparse
import os

REF_CUDA = {  # mpi/CUdata.txt:1-8 / makePlots.gp:17-19,29-31 (GB = 1e9 B)
    ("INT", "SUM"): 90.8413, ("INT", "MIN"): 90.7905, ("INT", "MAX"): 90.7969,
    ("DOUBLE", "SUM"): 92.7729, ("DOUBLE", "MIN"): 92.6014, ("DOUBLE", "MAX"): 92.7552,
}


def read_results(path):
    pts = []
    if not os.path.exists(path):
        return pts
    for line in open(path):
        p = line.split()
        if len(p) == 4:
            pts.append((int(p[2]), float(p[3])))
    return sorted(pts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--results", default="results")
    ap.add_argument("--out", default="plots")
    ap.add_argument("--reference-cuda", action="store_true", help="draw the reference CUDA constants")
    ap.add_argument("--single", default="", help="DT:OP=value,... single-GPU lines to draw")
    ap.add_argument("--ylabel", default="Bandwidth (GB/sec)")
    ap.add_argument("--label", default="MI355X", help="legend prefix of the measured series")
    ap.add_argument("--xlabel", default="Number of ranks (GPUs)")
    a = ap.parse_args()
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    os.makedirs(a.out, exist_ok=True)
    singles = {}
    for item in filter(None, a.single.split(",")):
        k, v = item.split("=")
        dt, op = k.split(":")
        singles[(dt, op)] = float(v)
    colors = {"MAX": "red", "MIN": "blue", "SUM": "green"}
    written = []
    for dt in ("INT", "DOUBLE", "LONG", "FLOAT"):
        series = {op: read_results(os.path.join(a.results, f"{dt}_{op}.txt")) for op in ("MAX", "MIN", "SUM")}
        if not any(series.values()):
            continue
        fig, ax = plt.subplots(figsize=(6, 4.5))
        for op, pts in series.items():
            if pts:
                ax.plot([p[0] for p in pts], [p[1] for p in pts], "-x", lw=2, color=colors[op], label=f"{a.label} {op}")
            if a.reference_cuda and (dt, op) in REF_CUDA:
                ax.axhline(REF_CUDA[(dt, op)], ls="--", lw=1.5, color=colors[op], label=f"ref CUDA {op}")
            if (dt, op) in singles:
                ax.axhline(singles[(dt, op)], ls=":", lw=2, color=colors[op], label=f"1 GPU {op}")
        ax.set_xlabel(a.xlabel)
        ax.set_ylabel(a.ylabel)
        ax.set_title({"INT": "Integers", "DOUBLE": "Doubles", "LONG": "int64", "FLOAT": "fp32"}[dt])
        ax.legend(loc="lower right", fontsize=8)
        path = os.path.join(a.out, f"{dt.lower()}.png")
        fig.tight_layout()
        fig.savefig(path, dpi=120)
        written.append(path)
    for p in written:
        print(p)


if __name__ == "__main__":
    main()
