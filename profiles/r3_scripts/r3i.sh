#!/bin/bash
# Round 3, GPU pass I: the whole GPU suite after the in-process-store change, smoke(), the driver's
# bench, and the fp32 window sweep (the HBM-fill config's element type).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
for n in 2e9 7.3e10; do
  timeout -k 10 300 ./build/bin/window_ab --type=float --n=$n --rounds=5 --iters=10 > $O/window_ab_f32_$n.txt 2>&1
  rc=$?; echo "window_ab_f32_$n rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
