#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_perf4
mkdir -p $O
for c in fused rccl; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-vector-extras --collective $c > $O/b_$c.json 2>/dev/null || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/p_$c -o t -- python bench.py --steps 100 --warmup 5 --no-vector-extras --no-serial-measure --collective $c > $O/p_$c.log 2>&1 || exit 1
done
for f in $O/b_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d.get('serial_gbps'))"; done
