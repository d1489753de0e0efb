#!/bin/bash
# Same-box kernel-only A/B (reduction app, hipEvent per iteration, 100 iterations, 8 GB float64 SUM):
# the round-1 tree (.ab/r1, ticketed tree fan-in) against this tree with the polled fan-in (default)
# and with MIREDUCE_FANIN=tree (round 1's fan-in), for the round-1 and round-3 8 GB plans.
O=${O:-gpurun_out/fanin_ab}
mkdir -p $O
cd "$GRAFT_REPO_ROOT"
run() {  # run <tag> <binary> <B> <U> <W>
  timeout -k 10 120 $2 --method=SUM --type=double --n=1e9 --fill=device --iterations=100 --threads=$3 --unroll=$4 \
      --wg-per-cu=$5 --noverify --log=none --master-log=none --json=$O/$1.jsonl > $O/$1.out 2>&1
  local rc=$?; echo "$1 rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) echo "stop $1 rc=$rc"; exit $rc;; esac
}
for r in 1 2 3; do
  for plan in "512 16 1" "256 8 1"; do
    set -- $plan
    tag="${1}x${2}x${3}"
    run r1_$tag .ab/r1/build/bin/reduction $1 $2 $3
    MIREDUCE_FANIN=poll run r3poll_$tag ./build/bin/reduction $1 $2 $3
    MIREDUCE_FANIN=tree run r3tree_$tag ./build/bin/reduction $1 $2 $3
  done
done
