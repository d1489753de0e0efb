#!/bin/bash
# Re-run of run8 after: a settle before each capture (NCCL watchdog), collective teardown of
# channels / direct buffers; then the auto-tune test once more and the kernel-time comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2_shard9
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_xrank_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { grep -v "frame #" $O/tests.log | tail -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread -p no:cacheprovider tests/test_xrank_gpu.py -k "tunes" > $O/tunes2.log 2>&1 || { grep -v "frame #" $O/tunes2.log | tail -30; exit 1; }
tail -1 $O/tunes2.log
bash profiles/r2_shard/run7.sh
