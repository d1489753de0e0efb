#!/bin/bash
# Round 4: cache-policy bits of the streaming body's buffer loads (kAuxNT): nt (shipped) vs sc0 nt,
# nt sc1, sc0 nt sc1 (build/ab_aux{3,18,19}: the same tree built with -DMIREDUCE_AUX=...). f64 SUM
# and bf16 SUM, 8 GB, default plans, same box, 3 interleaved rounds.
set -o pipefail
O=${O:-gpurun_out/r4_aux}
mkdir -p $O
one() {  # one <tag> <binary> <args...>
  local tag=$1 bin=$2; shift 2
  timeout -k 10 120 $bin "$@" --fill=device --iterations=60 --timing=batch --log=none \
      --master-log=none --json=$O/$tag.jsonl > $O/$tag.out 2>&1
  local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -3 $O/$tag.out; exit $rc; }
}
for r in 1 2 3; do
  for v in 2 3 18 19; do
    B=./build/ab_aux$v/reduction; [ $v = 2 ] && B=./build/bin/reduction
    one "f64_aux${v}_$r" $B --method=SUM --type=double --n=1e9
    one "bf16_aux${v}_$r" $B --method=SUM --type=bf16 --n=4e9
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[os.path.basename(f)[:-6].rsplit("_", 1)[0]].append((d["avg_ms"] * 1e3, d["gb_per_s"], d["verified"]))
for tag, v in sorted(acc.items()):
    print(f"{tag:14s} us {' '.join('%.2f' % x[0] for x in sorted(v)):28s} best GB/s {max(x[1] for x in v):8.1f} verified {all(x[2] for x in v)}")
PY
cat $O/summary.txt
