#!/bin/bash
# int64 MIN vs double SUM at 256M elements: operator or plan? (tools/op_ab.py)
set -o pipefail
mkdir -p gpurun_out/r5s
timeout -k 10 300 python -u tools/op_ab.py --n 268435456 --pairs float64:sum,int64:min,int64:max,int64:sum,float64:min \
  --variants "auto;xcd_skew=0;xcd_skew=20;window=2;unroll=4" --rounds 5 --json gpurun_out/r5s/op_ab.json \
  > gpurun_out/r5s/op_ab.txt 2>&1
