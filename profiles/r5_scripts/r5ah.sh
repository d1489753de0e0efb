#!/bin/bash
# the whole GPU suite on the last tree (test files changed since r5ab)
set -o pipefail
O=gpurun_out/r5ah
mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 $O/pytest_gpu.txt; exit $rc
