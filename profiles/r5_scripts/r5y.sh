#!/bin/bash
# bench.py's own timed windows split (MIREDUCE_WINDOW_PROBE=1) at the N=8 shard, K = 20 / 200, plan tuning on (the default)
set -o pipefail
O=gpurun_out/r5y
mkdir -p $O
export MIREDUCE_WINDOW_PROBE=1
for k in 20 200 20 200; do
  timeout -k 10 120 python3 bench.py --elements 125000000 --steps $k --warmup 5 --no-vector-extras --no-candidates \
    --extras-file $O/x.json > $O/k$k.json 2> $O/k$k.err || exit $?
  python3 -c "import json; d=json.load(open('$O/k$k.json')); print('K=$k ms_per_step', d['ms_per_step'])"
  grep "^\[window\]" $O/k$k.err
done | tee $O/summary.txt
