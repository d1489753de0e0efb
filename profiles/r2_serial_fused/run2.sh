#!/bin/bash
# After the chunked reduce.c verification: the 2-rank gloo capture-fallback bench with the extras,
# then every bench GPU test, then the default bench (serial measured with the fused finish).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_serial_fused
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_xrank_gpu.py tests/test_apps_gpu.py tests/test_fault_injection.py -m gpu -k "bench" -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests2.txt 2>&1 || { tail -40 $O/tests2.txt; exit 1; }
tail -2 $O/tests2.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
tail -1 $O/bench_default.err
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'], d['config']['collective'], d.get('serial_gbps'), d.get('serial_collective'), d.get('collective_tuning'))"
