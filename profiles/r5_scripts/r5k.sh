#!/bin/bash
# Round 5: does segmenting help below 16 GiB too? The 8 GB headline array (1e9 doubles) as one launch
# vs 1 / 2 / 4 GiB segments, and 32 / 64 GB arrays vs 4 / 8 / 16 GiB segments; 5 interleaved rounds,
# 10 back-to-back reductions per sample.
set -o pipefail
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 200 python3 tools/hbm_chunks.py --dtype float64 --elements 1e9 --rounds 5 --reps 10 --segments 1,2,4 --no-slices --no-stamps --json $O/seg_8g.jsonl > $O/seg_8g.txt 2>&1
rc=$?; echo "8g rc=$rc" >> $O/status.txt; grep "^\[hbm\]" $O/seg_8g.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/hbm_chunks.py --dtype float64 --elements 4e9 --rounds 5 --reps 3 --segments 4,8,16 --no-slices --no-stamps --json $O/seg_32g.jsonl > $O/seg_32g.txt 2>&1
rc=$?; echo "32g rc=$rc" >> $O/status.txt; grep "^\[hbm\]" $O/seg_32g.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/hbm_chunks.py --dtype float32 --elements 16e9 --rounds 3 --reps 2 --segments 4,8,16 --no-slices --no-stamps --json $O/seg_64g.jsonl > $O/seg_64g.txt 2>&1
rc=$?; echo "64g rc=$rc" >> $O/status.txt; grep "^\[hbm\]" $O/seg_64g.txt
exit $rc
