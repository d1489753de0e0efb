#!/bin/bash
# Round 3, GPU pass Z: the 32-192 MiB default (256x8x2 window 2): kernel GPU tests, and the
# reference's own default size (2^24 doubles) in the reduction app, new vs old plan, warm and cold.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_plan.py -m gpu -q -x --timeout 120 \
    --timeout-method thread > $O/pytest.out 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -2 $O/pytest.out
case $rc in 0) ;; *) exit $rc;; esac
B=./build/bin/reduction
C="--method=SUM --type=double --n=16777216 --fill=device --iterations=100 --log=none --master-log=none"
for r in 1 2 3; do
  for cold in "" "--cold"; do
    timeout -k 10 120 $B $C $cold --json=$O/ab.jsonl > /dev/null 2>> $O/ab.err; echo "new$cold rc=$?" >> $O/status.txt
    timeout -k 10 120 $B $C $cold --threads=256 --unroll=4 --wg-per-cu=3 --window=0 --json=$O/ab.jsonl > /dev/null 2>> $O/ab.err
    echo "old$cold rc=$?" >> $O/status.txt
  done
done
