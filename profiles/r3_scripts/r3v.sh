#!/bin/bash
# Round 3, GPU pass V: the fused-finish GPU tests again (pass U: the 8-rank shared-GPU rehearsal's
# direct DOUBLE SUM summary came back unverified; device errors are now reported), then every
# BASELINE config on the new self-check.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 300 python -u tools/settle_probe.py --json $O/settle_bf16.json > $O/settle_bf16.txt 2>&1
echo "settle_bf16 rc=$?" >> $O/status.txt
timeout -k 10 900 python -u -m pytest tests/test_xrank_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_xrank.out 2>&1
echo "pytest_xrank rc=$?" >> $O/status.txt
O=$O/configs bash tools/gpu/configs.sh > $O/configs_summary.txt 2>&1
echo "configs rc=$?" >> $O/status.txt
