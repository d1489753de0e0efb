#!/bin/bash
# Round 3, GPU pass Z (re-entry, fresh container rebuild): the whole GPU suite on HEAD (incl. the
# direct collective's CU split for ranks sharing a GPU and the device-side MAXLOC combine), smoke(),
# the driver's default bench, and rocprofv3 kernel stats of the default bench.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${PASS:-r3z}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc" >> $O/status.txt
case $rc in 0) ;; *) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err
echo "prof rc=$?" >> $O/status.txt
