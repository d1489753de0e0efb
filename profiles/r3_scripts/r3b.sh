#!/bin/bash
# Round 3, GPU pass B: r1-vs-r3 regression A/B, the HBM-fill investigation, and test_apps_gpu again.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/regress.sh || exit $?
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/hbmfill.sh || exit $?
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest tests/test_apps_gpu.py -v --timeout 300 --timeout-method thread \
    > gpurun_out/r3b/tests_apps.log 2>&1
echo "tests rc=$?" >> gpurun_out/r3b/status.txt
