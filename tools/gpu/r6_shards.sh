#!/bin/bash
# Round 6: the headline step at each N-GPU shard size, measured on one GPU (world 1: the same kernel,
# plan tuning and bound fused finish every rank of an N-GPU job runs, minus the xGMI exchange) with the
# driver's step window (K = 20, W = 5) and a long one (K = 200): the per-GPU column of the WRITEUP's
# scaling projection. 3 rounds, sizes interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r6_shards
mkdir -p $out
for r in 1 2 3; do
  for n in 1000000000 500000000 250000000 125000000; do
    for k in 20 200; do
      MIREDUCE_EXTRAS_DIR=$out timeout -k 10 240 python -u bench.py --steps $k --warmup 5 --elements $n \
        --no-vector-extras --no-candidates > $out/n${n}_k${k}_r$r.json 2> $out/n${n}_k${k}_r$r.err || exit $?
      echo "$n $k $r $(python -c "import json; d=[json.loads(l) for l in open('$out/n${n}_k${k}_r$r.json') if l.startswith('{')][0]; print(d['value'], d['ms_per_step'], d['verified'], d['summary'].get('plans'))")"
    done
  done
done
