#!/bin/bash
# Direct collective with U vectors per thread per trip for small worlds: direct GPU tests, then the
# default bench (reduce_c_vector.*_direct at N=1: 2 GiB in -> out through the W=1 kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_direct_unroll
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_apps_gpu.py tests/test_xrank_gpu.py tests/test_kernels_gpu.py -m gpu -k "direct or Direct" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'], json.dumps(d.get('reduce_c_vector')))"
