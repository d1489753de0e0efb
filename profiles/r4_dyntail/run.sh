#!/bin/bash
# Round 4 experiment: a workgroup-level dynamic tail (tools/dyntail_ab.hip) vs the production
# kernel with equal rounds and with the anchored XCD-weighted split; 1e9 doubles, same box.
O=gpurun_out/r4_dyntail
mkdir -p $O
timeout -k 10 240 ./build/bin/dyntail_ab --n=1e9 --rounds=5 --iters=20 > $O/dyntail_1e9_v2.txt 2>&1
echo "1e9 rc=$?" >> $O/status.txt
cat $O/dyntail_1e9_v2.txt
