#!/bin/bash
# New >= 3 GB plan for 8-byte types (256 x 8 x 1): plan/kernel GPU tests, then the default bench
# three times, the 4 GB shard (N=2) and the 256M int64 MIN config, each next to the old plan
# (--block 512 --unroll 16 --wg-per-cu 1) on the same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_plan4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_plan.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
OLD="--block 512 --unroll 16 --wg-per-cu 1"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-vector-extras > $O/new_default_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --no-vector-extras $OLD > $O/old_default_$r.json 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --no-vector-extras --steps 200 --warmup 20 --elements 500000000 > $O/new_4g.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --no-vector-extras --steps 200 --warmup 20 --elements 500000000 $OLD > $O/old_4g.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --no-vector-extras --config gpu_4g_bf16_sum > $O/new_bf16.json 2>/dev/null || exit 1
for f in $O/*.json; do python3 -c "import json; d=json.load(open('$f')); p=d['config']['kernel_plan']; print('$f', d['value'], d.get('serial_gbps'), p['block'], p['unroll'], p['grid'], d['verified'])"; done
