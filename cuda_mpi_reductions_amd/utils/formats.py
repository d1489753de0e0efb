"""Output formats of the reference, reproduced exactly.

* reduce.c GNUPlot lines (mpi/reduce.c:67-69,80-82,94-96): header ``# DATATYPE OP NODES GB/sec``,
  rows ``"%s %s %d %10.3lf"``, GB = 2^30 B of *total* data.
* CUDA-sample throughput line (cuda/C/src/reduction/reduction.cpp:744-745), GB = 1e9 B.

The C++ apps produce these lines through csrc/runtime/report.cpp; both implementations are tested
against each other and against the reference's own data files.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Iterable, Iterator

GIB = float(1 << 30)   # reduce.c's "GB" (mpi/reduce.c:79)
GB = 1.0e9             # reduction.cpp's "GB" (reduction.cpp:745)

GNUPLOT_HEADER = "# DATATYPE OP NODES GB/sec"
_ROW = re.compile(r"^(\S+) (\S+) (\d+)\s+(-?[0-9.]+)\s*$")
_THROUGHPUT = re.compile(
    r"^Reduction, Throughput = ([0-9.]+) GB/s, Time = ([0-9.]+) s, Size = (\d+) Elements, "
    r"NumDevsUsed = (\d+), Workgroup = (\d+)\s*$")


def gnuplot_line(dtype: str, op: str, nodes: int, gib_per_s: float) -> str:
    return "%s %s %d %10.3f" % (dtype, op, nodes, gib_per_s)


def throughput_line(gb_per_s: float, seconds: float, elements: int, num_devs: int, workgroup: int) -> str:
    return ("Reduction, Throughput = %.4f GB/s, Time = %.5f s, Size = %d Elements, NumDevsUsed = %d, "
            "Workgroup = %d" % (gb_per_s, seconds, elements, num_devs, workgroup))


@dataclass(frozen=True)
class Row:
    dtype: str
    op: str
    nodes: int
    value: float


def parse_gnuplot(lines: Iterable[str]) -> Iterator[Row]:
    """Rows of reduce.c-format output; comments and foreign lines are skipped."""
    for line in lines:
        m = _ROW.match(line.rstrip("\n"))
        if m:
            yield Row(m.group(1), m.group(2), int(m.group(3)), float(m.group(4)))


def parse_throughput(line: str):
    m = _THROUGHPUT.match(line.strip())
    if not m:
        return None
    return {"gb_per_s": float(m.group(1)), "seconds": float(m.group(2)), "elements": int(m.group(3)),
            "num_devs": int(m.group(4)), "workgroup": int(m.group(5))}
