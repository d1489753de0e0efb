#!/bin/bash
# Round 2: one-kernel direct collective (device-side barriers, graph replay) + auto/fused bench tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_direct
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_apps_gpu.py -k "direct" > $O/tests_direct.log 2>&1 &&
timeout -k 10 300 $T tests/test_xrank_gpu.py -k "auto" > $O/tests_auto.log 2>&1 &&
timeout -k 10 120 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?
grep -E "passed|failed|error" $O/tests_*.log | tail -5; cat $O/bench.json
exit $rc
