#!/bin/bash
# fp32 SUM (fp64 accumulation, the HBM-fill config's op) vs fp64 SUM and fp32 MAX at 2e9 / 1e9 elements
set -o pipefail
mkdir -p gpurun_out/r5u
timeout -k 10 300 python -u tools/op_ab.py --n 2000000000 --pairs float32:sum,float32:max,float64:sum \
  --variants "auto" --rounds 5 --reps 5 --json gpurun_out/r5u/op_ab_2e9.json > gpurun_out/r5u/op_ab_2e9.txt 2>&1
