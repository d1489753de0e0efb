#!/bin/bash
# 4-byte types from 3 GB: the current 512x4x1 against 256x8x1 / 256x4x2 / 256x2x3 (f32 SUM, i32 SUM, 8 GB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_plan5
mkdir -p $O
for spec in "float32 sum" "int32 sum"; do
  set -- $spec
  timeout -k 10 400 python -u tools/tune.py --dtype $1 --op $2 --ns 2000000000 --rounds 8 --iters 20 \
    --blocks 256,512 --unrolls 2,4,8 --wgs 1,2,3 --policies nt --top 8 > $O/h2h_$1.txt 2>&1 || { tail -20 $O/h2h_$1.txt; exit 1; }
  grep -v "^\[tune\]" $O/h2h_$1.txt
done
