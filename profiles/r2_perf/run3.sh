#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_perf3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_xrank_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-vector-extras"
for e in 125000000 250000000 500000000 1000000000; do
  $B --elements $e > $O/auto_$e.json 2>/dev/null || exit 1
done
timeout -k 10 120 python bench.py > $O/default.json 2> $O/default.err || exit 1
for f in $O/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d.get('serial_gbps'), d.get('collective_tuning'))"; done
