#!/bin/bash
# 1 GB shard, fused finish: stream lanes x graph chunk, interleaved repeats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2_shard4
mkdir -p $O
for rep in 1 2 3; do
  for cfg in "1 128" "2 128" "2 512" "3 512" "2 1000"; do
    set -- $cfg
    tag="s$1_c$2_r$rep"
    timeout -k 10 120 python bench.py --elements 125000000 --collective fused --streams $1 --graph-chunk $2 --steps 1000 --warmup 2 --no-vector-extras --no-serial-measure > $O/$tag.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'])"
  done
done
