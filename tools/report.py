#!/usr/bin/env python3
"""The reference's two report figures, redrawn with the MI355X results (docs/WRITEUP.md §2).

The reference's deliverable is two plots, ``int.eps`` and ``double.eps`` (mpi/makePlots.gp:1-40,
writeup.tex:21-29): BlueGene/L's element-wise MPI_Reduce bandwidth against the rank count (MAX /
MIN / SUM) with the single-GPU CUDA constants drawn across. This draws the same two figures and
puts on them everything this repo has measured in the same units:

* BG/L virtual-node mode (the reference's curves, tools/reference_data.py) — solid;
* the reference's CUDA constants (GT200/Fermi-class, kernel 6) — thin dashed;
* reduce.c rebuilt here on the build container's 8 CPUs (MPICH over shared memory, every run
  verified: profiles/r3_mpi_cpu/results/) — dotted, x = ranks;
* MI355X, one GPU reducing an array to one value (the reduction app / bench.py: ``--single``) —
  thick dashed horizontal;
* MI355X, reduce.c's own element-wise table on the node's GPUs (bench.py ``reduce_c_vector``, the
  one-kernel direct collective): the N = 1 value from a BENCH record (``--bench``) as a marker,
  and the N > 1 curve when a scaling run produced ``vector_direct/<DT>_<OP>.txt``
  (tools/scaling.py ``--from``; ``--vector``).

Units: every series in GB/s = 1e9 B/s; reduce.c's GiB/s values (BG/L, MPICH, the vector table) are
converted (x 2^30 / 1e9). Log-log axes (the series span 3.8 GB/s to 7.4 TB/s).

    python tools/report.py --out docs/figures [--single profiles/r6_single/single.json]
        [--bench BENCH_r06.json] [--vector results/scaling/vector_direct]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from reference_data import BGL_VN, CUDA, GIB_PER_GB  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS = ("MAX", "MIN", "SUM")
COLORS = {"MAX": "red", "MIN": "blue", "SUM": "green"}


def read_results(path: str) -> dict:
    """{ranks: value} from a getAvgs-format results file (``DT OP N value`` rows)."""
    pts = {}
    if os.path.exists(path):
        for line in open(path):
            p = line.split()
            if len(p) == 4:
                pts[int(p[2])] = float(p[3])
    return pts


def bench_vector_n1(path: str) -> dict:
    """{(DT, OP): GiB/s} of the direct reduce.c table in a BENCH record's (or bench line's)
    ``summary.reduce_c_rows`` (means over the retries; a ``!`` row failed verification: skipped)."""
    out = {}
    if not path or not os.path.exists(path):
        return out
    text = open(path).read()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from scaling import parse_text
    for r in parse_text(text):
        rows = ((r.get("summary") or {}).get("reduce_c_rows") or {}).get("direct")
        for item in str(rows or "").split(";"):
            p = item.split()
            if len(p) == 3 and not p[2].endswith("!"):
                out[(p[0], p[1])] = float(p[2])
    return out


def series(single: dict, bench: dict, vector_dir: str, mpich_dir: str) -> dict:
    """Every line of both figures, GB/s: {DT: [(label, style, {x: y} or scalar), ...]}."""
    out = {}
    for dt in ("INT", "DOUBLE"):
        s = []
        for op in OPS:
            s.append((f"BG/L VN {op}", ("-o", COLORS[op], 1.8),
                      {n: v / GIB_PER_GB for n, v in BGL_VN[(dt, op)].items()}))
        for op in OPS:
            pts = read_results(os.path.join(mpich_dir, f"{dt}_{op}.txt"))
            if pts:
                s.append((f"reduce.c, 8-CPU MPICH {op}", (":x", COLORS[op], 1.5),
                          {n: v / GIB_PER_GB for n, v in pts.items()}))
        for op in OPS:
            s.append((f"ref CUDA {op}", ("--", COLORS[op], 0.8), CUDA[(dt, op)]))
        for op in OPS:
            v = single.get(f"{dt} {op}")
            if v:
                s.append((f"MI355X 1 GPU {op}", ("-.", COLORS[op], 2.5), float(v["gbps"] if isinstance(v, dict) else v)))
        for op in OPS:
            pts = read_results(os.path.join(vector_dir, f"{dt}_{op}.txt")) if vector_dir else {}
            if (dt, op) in bench:
                pts.setdefault(1, bench[(dt, op)])
            if pts:
                s.append((f"MI355X reduce.c (direct) {op}", ("-s", COLORS[op], 2.5),
                          {n: v / GIB_PER_GB for n, v in pts.items()}))
        out[dt] = s
    return out


def draw(lines: dict, out_dir: str) -> list:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    os.makedirs(out_dir, exist_ok=True)
    written = []
    for dt, s in lines.items():
        fig, ax = plt.subplots(figsize=(8, 5.5))
        for label, (fmt, color, lw), data in s:
            if isinstance(data, dict):
                xs = sorted(data)
                ax.plot(xs, [data[x] for x in xs], fmt, color=color, lw=lw, ms=5, label=label)
            else:
                ax.axhline(data, ls=fmt, color=color, lw=lw, label=label)
        ax.set_xscale("log", base=2)
        ax.set_yscale("log")
        ax.set_xlim(0.8, 1400)
        ax.set_xlabel("Number of ranks (MPI ranks / GPUs)")
        ax.set_ylabel("Bandwidth (GB/s, 1e9 B/s)")
        ax.set_title({"INT": "Integers", "DOUBLE": "Doubles"}[dt] + ": MPI_Reduce vs one GPU, 2012 and MI355X")
        ax.grid(True, which="both", alpha=0.25)
        ax.legend(loc="center left", bbox_to_anchor=(1.01, 0.5), fontsize=7)
        path = os.path.join(out_dir, f"{dt.lower()}.png")
        fig.tight_layout()
        fig.savefig(path, dpi=110)
        plt.close(fig)
        written.append(path)
    return written


DEFAULT_SINGLE = os.path.join(ROOT, "profiles", "r6_single", "single.json")
DEFAULT_MPICH = os.path.join(ROOT, "profiles", "r3_mpi_cpu", "results")


def make_figures(out_dir: str, single_path: str = DEFAULT_SINGLE, bench_path: str = "", vector_dir: str = "",
                 mpich_dir: str = DEFAULT_MPICH) -> list:
    """Both figures into ``out_dir``; returns their paths."""
    single = json.load(open(single_path)) if single_path and os.path.exists(single_path) else {}
    return draw(series(single, bench_vector_n1(bench_path), vector_dir, mpich_dir), out_dir)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--out", default=os.path.join(ROOT, "docs", "figures"))
    ap.add_argument("--single", default=DEFAULT_SINGLE,
                    help='JSON {"INT SUM": {"gbps": ..., "source": ...}, ...}: one MI355X reducing an array')
    ap.add_argument("--bench", default="", help="a BENCH_r*.json / bench line: the N=1 reduce.c direct table")
    ap.add_argument("--vector", default="", help="dir with vector_direct/<DT>_<OP>.txt from a scaling run")
    ap.add_argument("--mpich", default=DEFAULT_MPICH)
    a = ap.parse_args(argv)
    for p in make_figures(a.out, a.single, a.bench, a.vector, a.mpich):
        print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
