#!/bin/bash
# Round 3, GPU pass E: the explicit in-flight-window experiment, then the whole GPU suite.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3e
mkdir -p $O
for n in 1e9 1.25e8; do
  timeout -k 10 300 ./build/bin/wg_timeline --set=window --n=$n --rounds=5 --iters=10 > $O/window_$n.txt 2>&1
  rc=$?; echo "window_$n rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt
tail -5 $O/pytest_gpu.log
