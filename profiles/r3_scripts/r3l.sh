#!/bin/bash
# Round 3, GPU pass L (fresh container, rebuilt tree): the whole GPU suite, smoke(), the driver's
# default bench, then pass K's sweeps (bf16/int32 windows) and every BASELINE.json GPU config.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
cat $O/bench_default.json
