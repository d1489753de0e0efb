#!/bin/bash
# Round 3, GPU pass W: the whole GPU suite on the current tree, smoke(), the driver's default bench,
# and the settle probe's new phases (G: release + 0.5 s idle; H: small-chunk torch pass + release).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${PASS:-r3w}
mkdir -p $O
timeout -k 10 300 python -u tools/settle_probe.py --json $O/settle_bf16.json > $O/settle_bf16.txt 2>&1
echo "settle rc=$?" >> $O/status.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo "bench rc=$?" >> $O/status.txt
