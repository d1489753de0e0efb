#!/bin/bash
# Round 4 final tree (XCD-anchored weighted split): the full GPU suite, smoke(), the default bench,
# a rocprofv3 kernel trace of the bench, then every BASELINE.json GPU config (tools/gpu/configs.sh).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${PASS:-r4_final}
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
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 \
    > $O/bench_prof.json 2> $O/bench_prof.err
rc=$?; echo "rocprof rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
O=$O/configs bash tools/gpu/configs.sh > $O/configs_summary.txt 2>&1
echo "configs rc=$?" >> $O/status.txt
