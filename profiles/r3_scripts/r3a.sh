#!/bin/bash
# Round 3, GPU pass A: the changed GPU tests, the driver's default bench, a rocprofv3 kernel trace.
set -o pipefail
O=gpurun_out/r3a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_fanin_gpu.py tests/test_xrank_gpu.py tests/test_apps_gpu.py \
    -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" | tee -a $O/status.txt
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo "bench rc=$?" | tee -a $O/status.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
    --no-vector-extras > $O/bench_prof.json 2> $O/bench_prof.err
echo "prof rc=$?" | tee -a $O/status.txt
