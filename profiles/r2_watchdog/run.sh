#!/bin/bash
# Extras watchdog: the deadline test and the bench GPU tests, then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_watchdog
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_xrank_gpu.py -m gpu -k "bench" -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'], d['config']['collective'], d['verified'], len(d['reduce_c_vector']['table']))"
