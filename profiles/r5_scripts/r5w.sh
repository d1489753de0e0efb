#!/bin/bash
# Fixed cost of the timed window at the N=8 shard (1 GB per GPU): ms_per_step at K = 20 / 50 / 200,
# interleaved, 3 rounds; t(K) = K * period + fixed.
set -o pipefail
O=gpurun_out/r5w
mkdir -p $O
for r in 1 2 3; do
  for k in 20 50 200; do
    timeout -k 10 120 python3 bench.py --elements 125000000 --steps $k --warmup 5 --no-vector-extras --no-candidates \
      --no-decompose --no-plan-tune --extras-file $O/x.json > $O/k${k}_r${r}.json 2> $O/k${k}_r${r}.err || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/k${k}_r${r}.json')); print('K=$k r=$r', d['ms_per_step'], d['verified'])"
  done
done | tee $O/summary.txt
