#!/bin/bash
# Reverted build (no sched_barrier). Which >= 3 GB plan for 8-byte types is robust across boxes:
# interleaved head-to-head at 8 GB (f64 SUM, int64 MAX) of 256x8x1, 256x16x1, 512x8x1, 512x16x1
# and 256x4x2, nt loads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_plan
mkdir -p $O
for spec in "float64 sum" "int64 max"; do
  set -- $spec
  timeout -k 10 400 python -u tools/tune.py --dtype $1 --op $2 --ns 1000000000 --rounds 10 --iters 20 \
    --blocks 256,512 --unrolls 8,16 --wgs 1 --policies nt > $O/h2h3_$1.txt 2>&1 || { tail -20 $O/h2h3_$1.txt; exit 1; }
  grep -v "^\[tune\]" $O/h2h3_$1.txt
done
