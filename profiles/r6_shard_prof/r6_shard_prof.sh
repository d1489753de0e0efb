#!/bin/bash
# Round 6, final tree: rocprofv3 kernel trace of the N=8 shard's step (1.25e8 doubles = 1 GB per GPU)
# run on one GPU through the driver's bench (K = 200 graph-replayed fused steps): per-launch time and
# the gaps between consecutive launches.
O=gpurun_out/r6_shard_prof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -o run -- \
  python3 bench.py --gpus 1 --elements 125000000 --steps 200 --warmup 5 --no-vector-extras > $O/bench.json 2> $O/bench.err || exit $?
python3 tools/prof_summary.py $O/raw > $O/kernel_stats.txt 2>&1
python3 tools/kernel_gaps.py $O/raw --match reduce_stream --bytes 1e9 > $O/gaps.txt 2>&1
rm -rf $O/raw
tail -1 $O/bench.json | head -c 300; echo; head -8 $O/kernel_stats.txt; tail -12 $O/gaps.txt
