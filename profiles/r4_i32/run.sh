#!/bin/bash
# Round 4 experiment: int32 SUM into int64 with dot2 half-sums (tools/i32sum_ab.hip) vs the
# production plans; 2e9 int32 (8 GB), same box.
O=gpurun_out/r4_i32
mkdir -p $O
timeout -k 10 300 ./build/bin/i32sum_ab --n=2e9 --rounds=5 --iters=20 > $O/i32sum_2e9_v2.txt 2>&1
echo "2e9 rc=$?" >> $O/status.txt
cat $O/i32sum_2e9_v2.txt
