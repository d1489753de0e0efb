#!/bin/bash
# Round 3, GPU pass AA: ranks sharing one GPU split its CUs for the direct collective's barrier
# kernel (pass U: the 8-rank rehearsal's direct DOUBLE SUM once came back unverified); the fused /
# direct GPU tests twice (the flaky case was 1 in 5).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3aa
mkdir -p $O
for r in 1 2; do
  timeout -k 10 900 python -u -m pytest tests/test_xrank_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread > $O/pytest_xrank_$r.out 2>&1
  rc=$?; echo "pytest_xrank_$r rc=$rc" >> $O/status.txt
  case $rc in 0|1) ;; *) exit $rc;; esac
done
