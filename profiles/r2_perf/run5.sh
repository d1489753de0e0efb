#!/bin/bash
# Re-measurement with committed outputs (the round-2 r2_perf runs only kept their scripts):
# the headline at every per-GPU shard of the N-GPU runs, auto-tuned combine, 200 steps; then the
# default bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_perf5
mkdir -p $O
B="timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-vector-extras"
for e in 125000000 250000000 500000000 1000000000; do
  $B --elements $e > $O/auto_$e.json 2>/dev/null || exit 1
done
timeout -k 10 120 python bench.py > $O/default.json 2> $O/default.err || exit 1
for f in $O/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config']['collective'], d['config']['streams'], d.get('serial_gbps'), d.get('collective_tuning',{}).get('gbps'))"; done
