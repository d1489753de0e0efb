#!/bin/bash
# the two round-4 GPU tests fixed after the first pass
O=gpurun_out/r4_tail
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  "tests/test_xrank_gpu.py::test_fused_poison_reaches_every_rank" \
  "tests/test_xrank_gpu.py::test_bench_fused_canary_two_ranks_one_gpu" \
  "tests/test_xrank_gpu.py::test_bench_torchrun_one_rank_graphs_both_modes" > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -le 1 ] || exit $rc
