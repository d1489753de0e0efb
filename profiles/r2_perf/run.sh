#!/bin/bash
# Per-GPU shard sizes of the N-GPU headline on one GPU: 1 GB (N=8), 2 GB (N=4), 4 GB (N=2), 8 GB (N=1);
# fused 1 lane / 2 lanes vs RCCL pipelined; plus kernel-only rocprof times at 1 GB and 128 MiB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_perf
mkdir -p $O
B="timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-vector-extras"
for e in 125000000 250000000 500000000; do
  $B --elements $e --collective fused > $O/fused1_$e.json 2>/dev/null || exit 1
  $B --elements $e --collective fused --streams 2 > $O/fused2_$e.json 2>/dev/null || exit 1
  $B --elements $e --collective rccl > $O/rccl_$e.json 2>/dev/null || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o sizes -- ./build/bin/reduction --method=SUM --type=double --n=125000000 --iterations=50 --log=none > $O/prof1g.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof128 -o sizes -- ./build/bin/reduction --method=SUM --type=double --n=16777216 --iterations=50 --log=none --cold > $O/prof128.log 2>&1
rc=$?
for f in $O/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d.get('serial_gbps'))"; done
exit $rc
