#!/bin/bash
# fp32 SUM (fp64 accumulation): plans with more waves per SIMD to hide the convert+add VALU work
set -o pipefail
mkdir -p gpurun_out/r5v
timeout -k 10 400 python -u tools/op_ab.py --n 2000000000 --pairs float32:sum,float64:sum \
  --variants "auto;wg_per_cu=2;wg_per_cu=3;wg_per_cu=2,window=2;block=512;block=512,window=2;unroll=4,window=4;unroll=4,window=4,wg_per_cu=2" \
  --rounds 4 --reps 5 --json gpurun_out/r5v/op_ab.json > gpurun_out/r5v/op_ab.txt 2>&1
