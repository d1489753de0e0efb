#!/bin/bash
# XCD skew vs array size for the 8-byte window-4 plan: the N=8 / 4 / 2 / 1 shards (1 / 2 / 4 / 8 GB)
set -o pipefail
mkdir -p gpurun_out/r5ak
for n in 125000000 250000000 500000000 1000000000; do
  reps=$((2000000000 / n * 10))
  timeout -k 10 400 python -u tools/op_ab.py --n $n --pairs float64:sum \
    --variants "xcd_skew=20;xcd_skew=30;xcd_skew=40;xcd_skew=50" --rounds 7 --reps $reps \
    --json gpurun_out/r5ak/skew_$n.json > gpurun_out/r5ak/skew_$n.txt 2>&1 || exit $?
  grep "^| float64" gpurun_out/r5ak/skew_$n.txt | sed "s/^/n=$n /"
done | tee gpurun_out/r5ak/summary.txt
