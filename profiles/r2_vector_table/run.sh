#!/bin/bash
# bench.py's reduce.c extras as the whole reduce.c table (INT/DOUBLE x MAX/MIN/SUM, RCCL + direct):
# the extras tests (1 rank nccl; 8 gloo ranks sharing the GPU), then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_vector_table
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_xrank_gpu.py -m gpu -k "extras_in_headline or eight_ranks_auto" -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value']);print('\n'.join(d['reduce_c_vector']['rows']))"
