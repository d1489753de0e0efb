#!/bin/bash
# Serial (per-reduction) measurement with the fused in-kernel finish whenever it passed its
# self-check: bench GPU tests, then the default bench, and an 8-rank rehearsal on the one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_serial_fused
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_xrank_gpu.py tests/test_apps_gpu.py -m gpu -k "bench" -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
tail -1 $O/bench_default.err
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'], d['config']['collective'], d.get('serial_gbps'), d.get('serial_collective'), d.get('collective_tuning'))"
