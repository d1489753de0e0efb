#!/bin/bash
# per-dispatch durations inside bench.py's timed windows at the N=8 shard (K=20), kernel trace only
O=gpurun_out/r5ao
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/kt -o run -- python3 bench.py --elements 125000000 --steps 20 --warmup 5 \
  --no-vector-extras --no-candidates --no-decompose --extras-file $O/x.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(find $O/kt -name "*.db" | head -1)
python3 tools/window_kernels.py "$db" --k 20 | tee $O/window_kernels.txt
rm -rf $O/kt
