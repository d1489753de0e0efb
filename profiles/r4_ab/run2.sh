#!/bin/bash
# Round 4: why did the reduction app measure XCD skew 20 slower than 0 (r4_ab) while bench.py and
# tools/xcd_balance.py measure it faster? Same process, same array, skews interleaved; then the
# array moved by one 32 KB tile (address-residue test); then the app with both fills.
set -o pipefail
O=${O:-gpurun_out/r4_ab2}
mkdir -p $O
timeout -k 10 240 python -u tools/xcd_balance.py --sizes 1000000000,125000000 --rounds 4 --launches 30 --skews 0,20 \
    --json $O/xcd_off0.jsonl > $O/xcd_off0.txt 2>&1
echo "xcd off0 rc=$?" >> $O/status.txt
timeout -k 10 240 python -u tools/xcd_balance.py --sizes 1000000000,125000000 --rounds 4 --launches 30 --skews 0,20 \
    --offset-tiles 1 --json $O/xcd_off1.jsonl > $O/xcd_off1.txt 2>&1
echo "xcd off1 rc=$?" >> $O/status.txt
one() {  # one <tag> <skew> <args...>
  local tag=$1; export MIREDUCE_XCD_SKEW=$2; shift 2
  timeout -k 10 120 ./build/bin/reduction --method=SUM --type=double --n=1e9 --fill=device --iterations=60 \
      --timing=batch --log=none --master-log=none --json=$O/$tag.jsonl "$@" > $O/$tag.out 2>&1
  local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
}
for r in 1 2 3; do
  for sk in 0 20; do
    one "app_small_s${sk}_$r" $sk
    one "app_unif_s${sk}_$r" $sk --pattern=uniform
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
O = sys.argv[1]
for f in ("xcd_off0.jsonl", "xcd_off1.jsonl"):
    acc = collections.defaultdict(list)
    for l in open(O + "/" + f):
        d = json.loads(l)
        acc[(d["n"], d["skew"])].append(d["us_per_launch"])
        base = d["base_mod_2mb"]
    for k, v in sorted(acc.items()):
        print(f, "n", k[0], "skew", k[1], "us", sorted(v), "base%2MB", base)
acc = collections.defaultdict(list)
for f in sorted(glob.glob(O + "/app_*.jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[os.path.basename(f)[:-6].rsplit("_", 1)[0]].append(d["avg_ms"] * 1e3)
for k, v in sorted(acc.items()):
    print(k, "us", ["%.2f" % x for x in sorted(v)])
PY
cat $O/summary.txt
