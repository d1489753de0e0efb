#!/bin/bash
# every plan-tuning candidate combined with the fused finish next to a rank of another plan
set -o pipefail
mkdir -p gpurun_out/r5aa
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xrank_gpu.py \
  -k "different_plans" > gpurun_out/r5aa/pytest.txt 2>&1
