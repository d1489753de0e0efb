#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_direct2
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_xrank_gpu.py -k "direct or extras" > $O/tests.log 2>&1 &&
timeout -k 10 120 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -5; cat $O/bench.json
exit $rc
