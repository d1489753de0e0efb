#!/bin/bash
# A/B of the new tuned default skew (2 rounds + 18 permille) against the old flat 20 permille
set -o pipefail
mkdir -p gpurun_out/r5al
for n in 125000000 250000000 500000000 1000000000; do
  reps=$((2000000000 / n * 10))
  timeout -k 10 400 python -u tools/op_ab.py --n $n --pairs float64:sum --variants "auto;xcd_skew=20" --rounds 9 \
    --reps $reps --json gpurun_out/r5al/f64_$n.json > gpurun_out/r5al/f64_$n.txt 2>&1 || exit $?
  grep "^| float64" gpurun_out/r5al/f64_$n.txt | sed "s/^/n=$n /"
done | tee gpurun_out/r5al/summary.txt
timeout -k 10 400 python -u tools/op_ab.py --n 268435456 --pairs int64:min,float64:max --variants "auto;xcd_skew=20" \
  --rounds 7 --reps 40 --json gpurun_out/r5al/cfg3.json > gpurun_out/r5al/cfg3.txt 2>&1 &&
grep "^| " gpurun_out/r5al/cfg3.txt | tee -a gpurun_out/r5al/summary.txt
