#!/bin/bash
# reduce.hip split into reduce_kernels.hpp + eight reduce_tab_*.hip TUs: streaming-kernel GPU tests,
# smoke, and the default bench on the rebuilt tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_split
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_ops.py tests/test_half.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
cat $O/bench_default.json
