#!/bin/bash
# Round 4: do the plans that reject a positive XCD skew (bf16 SUM window 4, int32 SUM window 2 at
# 2 WG/CU) want a negative one (extra rounds on the even XCCs)? Reduction app, 8 GB, 2 rounds.
set -o pipefail
O=${O:-gpurun_out/r4_skew2}
mkdir -p $O
one() {  # one <tag> <skew> <args...>
  local tag=$1; export MIREDUCE_XCD_SKEW=$2; shift 2
  timeout -k 10 120 ./build/bin/reduction "$@" --fill=device --iterations=60 --timing=batch --log=none \
      --master-log=none --json=$O/$tag.jsonl > $O/$tag.out 2>&1
  local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -3 $O/$tag.out; exit $rc; }
}
for r in 1 2; do
  for sk in 0 -10 -20 -30 5; do
    one "i32sum_s${sk}_$r" $sk --method=SUM --type=int --n=2e9
    one "bf16sum_s${sk}_$r" $sk --method=SUM --type=bf16 --n=4e9
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[os.path.basename(f)[:-6].rsplit("_", 1)[0]].append((d["avg_ms"] * 1e3, d["gb_per_s"], d["verified"], d["window"], d["grid"]))
for tag, v in sorted(acc.items()):
    print(f"{tag:14s} us {' '.join('%.2f' % x[0] for x in sorted(v)):28s} best GB/s {max(x[1] for x in v):8.1f} "
          f"verified {all(x[2] for x in v)} window {v[0][3]} grid {v[0][4]}")
PY
cat $O/summary.txt
