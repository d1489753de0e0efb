#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_c6
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_apps_gpu.py -k "multipass or threads_reference or huge or bandwidth or reduce_xgmi_single_rank or scalar_corrupt or every_kernel or app_paths" > $O/tests.log 2>&1
rc=$?
./build/bin/bandwidth_test --size=1G --iters=10 > $O/bandwidth.txt 2>&1
grep -E "passed|failed|error" $O/tests.log | tail -5
exit $rc
