#!/bin/bash
# Round 4 same-box A/B: the reduction app built from the tree just before the TileSeq window body
# (build/ab_pre/reduction, commit bc59f54) vs the current tree, kernel-only (batch timing, 60
# iterations), interleaved 3 rounds: int32 SUM (window 2, 2 WG/CU), bf16 SUM and f64 SUM (window 4;
# skew 0 to compare the body alone, and the default).
set -o pipefail
O=${O:-gpurun_out/r4_ab}
mkdir -p $O
one() {  # one <tag> <binary> <skew or ''> <args...>
  local tag=$1 bin=$2 sk=$3; shift 3
  if [ -n "$sk" ]; then export MIREDUCE_XCD_SKEW=$sk; else unset MIREDUCE_XCD_SKEW; fi
  timeout -k 10 120 $bin "$@" --fill=device --iterations=60 --timing=batch --log=none --master-log=none \
      --json=$O/$tag.jsonl > $O/$tag.out 2>&1
  local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -3 $O/$tag.out; exit $rc; }
}
for r in 1 2 3; do
  for v in pre cur; do
    B=./build/bin/reduction; [ $v = pre ] && B=./build/ab_pre/reduction
    one "i32_${v}_$r" $B 0 --method=SUM --type=int --n=2e9
    one "bf16_${v}_$r" $B 0 --method=SUM --type=bf16 --n=4e9
    one "f64_${v}_s0_$r" $B 0 --method=SUM --type=double --n=1e9
    [ $v = cur ] && one "f64_${v}_def_$r" $B "" --method=SUM --type=double --n=1e9
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[os.path.basename(f)[:-6].rsplit("_", 1)[0]].append((d["avg_ms"] * 1e3, d["gb_per_s"], d["verified"]))
for tag, v in sorted(acc.items()):
    print(f"{tag:14s} us {' '.join('%.2f' % x[0] for x in sorted(v)):32s} best GB/s {max(x[1] for x in v):8.1f} verified {all(x[2] for x in v)}")
PY
cat $O/summary.txt
