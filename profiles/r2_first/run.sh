#!/bin/bash
# Round 2, first GPU pass: new xrank/bench tests, smoke, bench (rccl + fused), rocprof kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_first
mkdir -p $O
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_xrank_gpu.py tests/test_arg_reduce.py -k "xrank or fused or bench or split_scratch" > $O/tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench_rccl.json 2> $O/bench_rccl.err &&
timeout -k 10 300 python bench.py --collective fused > $O/bench_fused.json 2> $O/bench_fused.err &&
timeout -k 10 300 python bench.py --collective fused --streams 2 > $O/bench_fused2.json 2> $O/bench_fused2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rccl -o run -- python bench.py --steps 20 --warmup 3 > $O/prof_rccl.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fused -o run -- python bench.py --steps 20 --warmup 3 --collective fused > $O/prof_fused.log 2>&1
rc=$?
tail -3 $O/tests.log; cat $O/bench_*.json
exit $rc
