#!/bin/bash
# Full GPU suite (with the 25 slowest tests listed) + smoke + default bench on the tree at the end of round 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_final6
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --durations=25 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.log 2>&1
rc=$?
tail -32 $O/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -1 $O/smoke.log; cat $O/bench.json
exit $rc
