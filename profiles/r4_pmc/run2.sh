#!/bin/bash
# Round 4: the PMC pass (isolated, serialised launches) read skew 20 as 1.4 % longer in GPU-active
# cycles than skew 0, while back-to-back timing reads it 0.5 % faster. Timing by launch shape:
# batch (back-to-back, one event pair), per-iter (an event pair per launch), --cold (1 GiB flush
# kernel between launches); f64 SUM 8 GB, skew 0 / 20, 3 interleaved rounds.
set -o pipefail
O=${O:-gpurun_out/r4_pmc2}
mkdir -p $O
one() {  # one <tag> <skew> <args...>
  local tag=$1; export MIREDUCE_XCD_SKEW=$2; shift 2
  timeout -k 10 120 ./build/bin/reduction --method=SUM --type=double --n=1e9 --fill=device --log=none \
      --master-log=none --json=$O/$tag.jsonl "$@" > $O/$tag.out 2>&1
  local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -3 $O/$tag.out; exit $rc; }
}
for r in 1 2 3; do
  for sk in 0 20; do
    one "batch_s${sk}_$r" $sk --iterations=60 --timing=batch
    one "periter_s${sk}_$r" $sk --iterations=60 --timing=per-iter
    one "cold_s${sk}_$r" $sk --iterations=30 --cold
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections, statistics
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[os.path.basename(f)[:-6].rsplit("_", 1)[0]].append((d["avg_ms"] * 1e3, d["median_ms"] * 1e3, d["verified"]))
for tag, v in sorted(acc.items()):
    print(f"{tag:14s} avg us {' '.join('%.2f' % x[0] for x in sorted(v)):26s} median us {' '.join('%.2f' % x[1] for x in sorted(v, key=lambda x: x[1])):26s} verified {all(x[2] for x in v)}")
PY
cat $O/summary.txt
