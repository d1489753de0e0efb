#!/bin/bash
# Round 5, session 1: the GPU suite after the bench restructure and the late-anchor fix, then the
# driver's bench command (N=1) and its sidecar.
set -o pipefail
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc" | tee $O/status.txt
tail -5 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --extras-file $O/bench_extras_n1.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc" | tee -a $O/status.txt; cat $O/bench.json
exit $rc
