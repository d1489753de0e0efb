#!/bin/bash
# Round 3, GPU pass Y: do the explicit-window plans also win below 192 MB (the reference's default
# 2^24 doubles = 128 MiB, and 32 / 64 MiB)? f64 and f32 SUM, interleaved rounds.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3y
mkdir -p $O
for spec in "float64 16777216" "float64 8388608" "float64 4194304" "float32 33554432" "float64 25165824"; do
  set -- $spec
  timeout -k 10 300 python -u tools/tune.py --dtype $1 --n $2 --blocks 256,512 --unrolls 2,4,8 --wgs 1,2,3,4 \
      --policies nt --windows 0,2,4 --rounds 7 --iters 50 --json $O/tune_$1_$2.json > $O/tune_$1_$2.txt 2>&1
  rc=$?; echo "tune_$1_$2 rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
