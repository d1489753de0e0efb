#!/bin/bash
# the line's new fields: config.collective_reason after a fallback, summary.wait_us / config.peer_access at N=8
set -o pipefail
mkdir -p gpurun_out/r5ac
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xrank_gpu.py \
  -k "remeasures or eight_ranks" > gpurun_out/r5ac/pytest.txt 2>&1
