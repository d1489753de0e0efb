#!/usr/bin/env bash
# Format-compatible replacement for the reference's mpi/getAvgs.sh:3-14: reads reduce.c-format
# lines ("DATATYPE OP NODES GB/sec") from a collected file and writes results/<DT>_<OP>.txt with
# bc-style scale=5 averages per rank count. Implemented in cuda_mpi_reductions_amd.utils.getavgs
# (bc is not installed on every box).
#   usage: tools/getAvgs.sh [collected.txt] [results_dir]
set -euo pipefail
HERE="$(cd "$(dirname "$0")/.." && pwd)"
COLLECTED="${1:-collected.txt}"
RESULTS="${2:-results}"
PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}" python3 -m cuda_mpi_reductions_amd.utils.getavgs "$COLLECTED" "$RESULTS"
