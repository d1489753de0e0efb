#!/bin/bash
# where does the ~2.4 us fixed cost of the 1 GB shard kernel go?
#  A. quantisation: 1 GB (30517 tiles = 119.2 rounds) vs exactly 119 and 120 whole rounds
#  B. balanced leftover, prefetched before the body (MIREDUCE_BALANCE=1) vs the default, 1 GB + 8 GB
#  C. the floor: a tiny array through the same headline protocol
#  D. the fused finish's cost per step: headline vs the same kernel without the channel (decomposition)
# bench.py headline protocol (serial, graph-replayed, fused finish), plan tuning off; interleaved.
set -o pipefail
O=${O:-gpurun_out/r4_tail}
mkdir -p $O
run() {  # run <tag> <env> <elements> <steps>
  env $2 timeout -k 10 180 python -u bench.py --elements $3 --steps $4 --warmup 10 --no-vector-extras --no-candidates \
      --no-plan-tune > $O/$1.json 2> $O/$1.err
  local rc=$?; echo "$1 rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || { tail -5 $O/$1.err; exit $rc; }
}
for r in 1 2 3; do
  for n in 124780544 125000000 125829120; do
    run "n${n}_def_$r" "MIREDUCE_BALANCE=0" $n 400
    run "n${n}_bal_$r" "MIREDUCE_BALANCE=1" $n 400
  done
  run "n1e9_def_$r" "MIREDUCE_BALANCE=0" 1000000000 60
  run "n1e9_bal_$r" "MIREDUCE_BALANCE=1" 1000000000 60
done
run "tiny_def" "MIREDUCE_BALANCE=0" 1024 400
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(O + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    tag = os.path.basename(f)[:-5].rsplit("_", 1)[0]
    dec = d.get("decomposition") or {}
    acc[tag].append((d["ms_per_step"] * 1e3, d["value"], d["verified"], dec.get("local_ms_per_step", 0) * 1e3,
                     (dec.get("exchange_wait_us") or {}).get("min_rank_median")))
for tag, v in sorted(acc.items()):
    us = sorted(x[0] for x in v)
    loc = sorted(x[3] for x in v)
    print(f"{tag:24s} us/step {' '.join('%.2f' % u for u in us):30s} local {' '.join('%.2f' % u for u in loc):30s} "
          f"GB/s {max(x[1] for x in v):9.1f} verified {all(x[2] for x in v)} wait {v[0][4]}")
PY
cat $O/summary.txt
