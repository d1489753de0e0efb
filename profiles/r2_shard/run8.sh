#!/bin/bash
# After prefetching the fused finish's descriptor fields before the finisher polls: fused/xrank and
# kernel numerics tests, then the local / rccl / fused kernel-time comparison (run7.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2_shard8
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_xrank_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash profiles/r2_shard/run7.sh
