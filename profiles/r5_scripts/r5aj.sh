#!/bin/bash
# finer XCD-skew grid for the 8 GB headline plan (permille: 0 / 10 / 20 (default) / 30 / 40), interleaved
set -o pipefail
mkdir -p gpurun_out/r5aj
timeout -k 10 400 python -u tools/op_ab.py --n 1000000000 --pairs float64:sum \
  --variants "auto;xcd_skew=0;xcd_skew=10;xcd_skew=20;xcd_skew=30;xcd_skew=40" --rounds 7 --reps 10 \
  --json gpurun_out/r5aj/skew.json > gpurun_out/r5aj/skew.txt 2>&1 &&
timeout -k 10 400 python -u tools/op_ab.py --n 125000000 --pairs float64:sum \
  --variants "auto;xcd_skew=0;xcd_skew=10;xcd_skew=20;xcd_skew=30;xcd_skew=40" --rounds 7 --reps 50 \
  --json gpurun_out/r5aj/skew_1g.json > gpurun_out/r5aj/skew_1g.txt 2>&1
