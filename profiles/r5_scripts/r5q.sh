#!/bin/bash
# RCCL re-measure fallback when the fused finish fails the headline steps (ranks share the GPU)
set -o pipefail
mkdir -p gpurun_out/r5q
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xrank_gpu.py \
  -k "fused_corrupt or remeasures or eight_ranks_auto" > gpurun_out/r5q/pytest.txt 2>&1
