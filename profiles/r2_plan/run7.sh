#!/bin/bash
# Per-run plan choice in bench.py (--collective auto measures the tuned default against the
# runners-up for the 8-byte headline shards): bench GPU tests, then the default bench and the
# 1 GB shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_plan7
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_xrank_gpu.py tests/test_apps_gpu.py -m gpu -k "bench" -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
s=$SECONDS
timeout -k 10 300 python bench.py > $O/default.json 2> $O/default.err || exit $?
echo "default bench wall $((SECONDS - s)) s"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --elements 125000000 --no-vector-extras > $O/shard_1g.json 2> $O/shard_1g.err || exit $?
for f in $O/*.json; do python3 -c "import json; d=json.load(open('$f')); p=d['config']['kernel_plan']; print('$f', d['value'], d.get('serial_gbps'), p['block'], p['unroll'], p['grid'], d.get('plan_tuning'), d['config']['collective'], d['verified'])"; done
