#!/bin/bash
# Serial number measured with both combines (fused finish and RCCL) when the fused finish works:
# bench GPU tests, then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_serial_fused
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_xrank_gpu.py tests/test_apps_gpu.py -m gpu -k "bench" -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests3.txt 2>&1 || { tail -40 $O/tests3.txt; exit 1; }
tail -1 $O/tests3.txt
timeout -k 10 300 python bench.py > $O/bench_default3.json 2> $O/bench_default3.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_default3.json'));print(d['value'], d['config']['collective'], d.get('serial_gbps'), d.get('serial_collective'), d.get('serial_candidates_gbps'), d.get('collective_tuning'))"
