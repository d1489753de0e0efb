#!/bin/bash
# Follow-up of r6_ladder.sh: ladder kernel 6 (whitepaper kernel 7) is capped at the reference's 64
# blocks (reduction.cpp's maxBlocks), sized for G80's 16 SMs; here with the grid scaled to MI355X's
# 256 CUs (--maxblocks 256 / 1024 / 2048), 128 threads as in the whitepaper.
O=gpurun_out/r6_ladder; mkdir -p $O
cd "$GRAFT_REPO_ROOT"
for n in 4194304 33554432; do
  for mb in 64 256 1024 2048; do
    for mode in warm cold; do
      c=""; [ $mode = cold ] && c="--cold"
      f=$O/k6mb${mb}_n${n}_${mode}
      timeout -k 10 120 ./build/bin/reduction --method=SUM --type=int --n=$n --kernel=6 --threads=128 --maxblocks=$mb $c \
        --iterations=100 --log=none --master-log=none --json=$f.json > $f.txt 2>&1 || exit $?
      echo "n=$n k=6 maxblocks=$mb $mode: $(grep -h -i "throughput" $f.txt | head -1)"
    done
  done
done
