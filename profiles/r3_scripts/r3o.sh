#!/bin/bash
# Round 3, GPU pass O: explicit-window sweeps for the 4-byte and 2-byte element types at 8 GB
# (window_ab showed 256x8x1 window 4 ahead of the 4-byte default 512x4x1 for f32 at 8 GB and 292 GB,
# profiles/r3_pass_i/): int32 SUM (int64 acc), f32 SUM, bf16 SUM, interleaved rounds, one process each.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3o
mkdir -p $O
for spec in "int32 2e9" "float32 2e9" "bfloat16 4e9" "int32 5e8" "float32 5e8"; do
  set -- $spec
  timeout -k 10 400 python -u tools/tune.py --dtype $1 --n $2 --blocks 256,512 --unrolls 2,4,8 --wgs 1,2,3 \
      --policies nt --windows 0,2,4 --rounds 5 --iters 10 --json $O/tune_$1_$2.json > $O/tune_$1_$2.txt 2>&1
  rc=$?; echo "tune_$1_$2 rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
