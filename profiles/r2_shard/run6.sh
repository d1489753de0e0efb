#!/bin/bash
# Kernel trace of the 1 GB-shard bench, fused finish, 1 vs 2 stream lanes: per-kernel time and the
# steady-state period / overlap of the timed graph (tools/prof_db.py --steady).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_shard6
mkdir -p $O
for s in 1 2; do
  timeout -k 10 180 rocprofv3 --kernel-trace -d $O/p$s -o t -- python bench.py --elements 125000000 --collective fused --streams $s --steps 300 --warmup 5 --no-serial-measure --no-vector-extras > $O/bench_s$s.json 2> $O/bench_s$s.err || { tail -5 $O/bench_s$s.err; exit 1; }
  db=$(ls $O/p$s/*/t_results.db $O/p$s/t_results.db 2>/dev/null | head -1)
  python tools/prof_db.py "$db" --steady reduce_stream > $O/lanes_$s.txt && rm -rf $O/p$s
  echo "== $s lane(s)"; cat $O/lanes_$s.txt; tail -1 $O/bench_s$s.json | cut -c1-200
done
