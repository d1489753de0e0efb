#!/bin/bash
# Kernel time of the 1 GB-shard step kernel: local only vs RCCL combine vs fused finish (1 lane).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_shard7
mkdir -p $O
for mode in local rccl fused local2; do
  case $mode in
    local|local2) extra="--local-only";;
    *) extra="--collective $mode";;
  esac
  timeout -k 10 180 rocprofv3 --kernel-trace -d $O/p_$mode -o t -- python bench.py --elements 125000000 $extra --steps 300 --warmup 5 --no-serial-measure --no-vector-extras > $O/bench_$mode.json 2> $O/bench_$mode.err || { tail -5 $O/bench_$mode.err; exit 1; }
  db=$(ls $O/p_$mode/*/t_results.db $O/p_$mode/t_results.db 2>/dev/null | head -1)
  python tools/prof_db.py "$db" --steady reduce_stream > $O/k_$mode.txt && rm -rf $O/p_$mode
  echo "== $mode"; grep -E "reduce_stream|steady" $O/k_$mode.txt
done
