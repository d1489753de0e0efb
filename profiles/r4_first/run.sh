#!/bin/bash
# Round 4 first GPU pass: the new GPU tests (identity poison, check=True, epoch wrap, cross-rank
# poison propagation, native peer preflight, replay probe, decomposition), smoke, default bench.
set -o pipefail
O=gpurun_out/r4_first
mkdir -p $O
timeout -k 10 840 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_fanin_gpu.py tests/test_xrank_gpu.py::test_fused_poison_reaches_every_rank \
  tests/test_xrank_gpu.py::test_fused_missing_peer_times_out_not_hangs \
  tests/test_xrank_gpu.py::test_bench_replay_probe_and_decomposition_one_gpu \
  tests/test_xrank_gpu.py::test_bench_replay_probe_failure_goes_eager_one_gpu \
  tests/test_xrank_gpu.py::test_fused_world1_matches_torch \
  tests/test_xrank_gpu.py::test_bench_torchrun_one_rank_graphs_both_modes \
  tests/test_xrank_gpu.py::test_bench_fused_canary_two_ranks_one_gpu \
  tests/test_xrank_gpu.py::test_bench_fused_ranks_share_one_gpu \
  tests/test_apps_gpu.py::test_reduce_xgmi_peer_preflight_declines_on_every_rank \
  tests/test_apps_gpu.py::test_reduce_xgmi_scalar_fused > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" > $O/status.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
