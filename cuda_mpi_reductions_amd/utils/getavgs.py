"""Averaging of reduce.c-format results — a re-implementation of mpi/getAvgs.sh:3-14.

For each DATATYPE in (INT, DOUBLE) and OP in (SUM, MIN, MAX) the script writes
``results/<DT>_<OP>.txt``: a blank first line, then one ``"<DT> <OP> <NODES> <AVG>"`` line per
rank count (rank counts sorted numerically, ``sort -n | uniq``), where AVG is the mean of column 4
printed with bc's ``scale=5`` (truncated, not rounded, to 5 decimals). Extended dtypes (LONG,
FLOAT) are included when present. Usage:

    python -m cuda_mpi_reductions_amd.utils.getavgs collected.txt results/
"""
from __future__ import annotations

import os
import sys
from collections import OrderedDict
from decimal import ROUND_DOWN, Decimal
from typing import Dict, Iterable, List, Tuple

from .formats import parse_gnuplot

DTYPES = ("INT", "DOUBLE")
EXTRA_DTYPES = ("LONG", "FLOAT")
OPS = ("SUM", "MIN", "MAX")


def bc_div(total: str, count: int) -> str:
    """``echo "scale=5; total / count" | bc`` — truncation toward zero, bc's output style."""
    q = (Decimal(total) / Decimal(count)).quantize(Decimal("0.00001"), rounding=ROUND_DOWN)
    s = format(q, "f")
    if s.startswith("0."):
        s = s[1:]          # bc prints ".12345" for values below 1
    elif s.startswith("-0."):
        s = "-" + s[2:]
    return s


def awk_sum(values: List[str]) -> str:
    """awk '{ sum += $4 } END { print sum }' uses %.6g output formatting."""
    total = sum(float(v) for v in values)
    return "%.6g" % total


def averages(lines: Iterable[str]) -> Dict[Tuple[str, str], List[Tuple[int, str]]]:
    raw: Dict[Tuple[str, str, int], List[str]] = OrderedDict()
    for line in lines:
        parts = line.split()
        if len(parts) < 4 or line.startswith("#"):
            continue
        try:
            nodes = int(parts[2])
            float(parts[3])
        except ValueError:
            continue
        raw.setdefault((parts[0], parts[1], nodes), []).append(parts[3])
    out: Dict[Tuple[str, str], List[Tuple[int, str]]] = {}
    for (dt, op, nodes), vals in raw.items():
        out.setdefault((dt, op), []).append((nodes, bc_div(awk_sum(vals), len(vals))))
    for k in out:
        out[k].sort(key=lambda t: t[0])
    return out


def write_results(collected_path: str, results_dir: str) -> List[str]:
    with open(collected_path) as f:
        avgs = averages(f.readlines())
    os.makedirs(results_dir, exist_ok=True)
    written = []
    dts = list(DTYPES) + [d for d in EXTRA_DTYPES if any(k[0] == d for k in avgs)]
    for dt in dts:
        for op in OPS:
            path = os.path.join(results_dir, f"{dt}_{op}.txt")
            with open(path, "w") as f:
                f.write("\n")
                for nodes, avg in avgs.get((dt, op), []):
                    f.write(f"{dt} {op} {nodes} {avg}\n")
            written.append(path)
    return written


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 2:
        print(__doc__)
        return 2
    for p in write_results(argv[0], argv[1]):
        print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
