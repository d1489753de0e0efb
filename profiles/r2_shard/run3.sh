#!/bin/bash
# Why does the 2-lane fused headline at 1 GB measure lower than its tuning run? Steps / chunk sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2_shard3
mkdir -p $O
for args in "--steps 210 --warmup 2" "--steps 400 --warmup 40" "--steps 400 --warmup 2" "--steps 1000 --warmup 2" "--steps 400 --warmup 2 --graph-chunk 400" "--steps 210 --warmup 2"; do
  for s in 1 2; do
    tag=$(echo "s$s $args" | tr ' -' '__')
    timeout -k 10 120 python bench.py --elements 125000000 --collective fused --streams $s --no-vector-extras --no-serial-measure $args > $O/$tag.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['config'].get('launch', d.get('launch')))"
  done
done
