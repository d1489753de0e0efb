#!/bin/bash
# A/B: the polled fan-in's finisher with two poll rounds in flight (MIREDUCE_POLL_PIPE=1) vs one.
# launch_floor (graph-replayed back-to-back launches; fan-in alone, 2^24 doubles, the 1 GB shard),
# 3 interleaved pairs; then the fan-in GPU tests with the knob on.
set -o pipefail
O=gpurun_out/r5ae
mkdir -p $O
for r in 1 2 3; do
  for p in 0 1; do
    MIREDUCE_POLL_PIPE=$p timeout -k 10 180 ./build/bin/launch_floor --rounds=5 --launches=200 > $O/floor_p${p}_r${r}.txt 2>&1
    rc=$?; echo "pipe=$p round=$r rc=$rc"; [ $rc -le 1 ] || exit $rc
    grep -E "poll768 |reduce_16777216 |reduce_125000000 |empty768 " $O/floor_p${p}_r${r}.txt | sed "s/^/pipe=$p r=$r /"
  done
done | tee $O/summary.txt
MIREDUCE_POLL_PIPE=1 timeout -k 10 600 python3 -u -m pytest tests/test_fanin_gpu.py tests/test_kernels_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest_pipe.txt 2>&1
rc=$?; echo "pytest pipe=1 rc=$rc"; tail -2 $O/pytest_pipe.txt; exit $rc
