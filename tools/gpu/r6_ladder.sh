#!/bin/bash
# The Harris whitepaper's table (2^22 int32 SUM, 128 threads per block, kernels 1-7 =
# this repo's ladder kernels 0-6) redrawn on one MI355X through the reduction app, plus mireduce's
# own single-pass kernel (7, tuned plan) — warm (array in the 256 MB Infinity Cache / L2) and cold
# (--cold: HBM), and the whitepaper's 32M-element point.
O=gpurun_out/r6_ladder; mkdir -p $O
cd "$GRAFT_REPO_ROOT"
for n in 4194304 33554432; do
  for k in 0 1 2 3 4 5 6 7; do
    th="--threads=128"; [ $k = 7 ] && th=""
    for mode in warm cold; do
      c=""; [ $mode = cold ] && c="--cold"
      timeout -k 10 120 ./build/bin/reduction --method=SUM --type=int --n=$n --kernel=$k $th $c --iterations=100 \
        --log=none --master-log=none --json=$O/k${k}_n${n}_${mode}.json > $O/k${k}_n${n}_${mode}.txt 2>&1 || exit $?
      echo "n=$n k=$k $mode: $(grep -h -i "throughput" $O/k${k}_n${n}_${mode}.txt | head -1)"
    done
  done
done
