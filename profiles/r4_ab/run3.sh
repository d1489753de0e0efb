#!/bin/bash
# Round 4: (1) the incremental 32-bit TileSeq walker vs the pre-TileSeq build (same box, skew 0),
# (2) does the blockIdx -> XCC deal depend on the stream (hardware queue)? (3) the XCD-anchored split
# (XcdAnchor) at skew +-20 in the app. The reduction app (own
# non-blocking stream) measured skew 20 slower, tools/xcd_balance.py (torch's current stream) faster.
set -o pipefail
O=${O:-gpurun_out/r4_ab3}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_fanin_gpu.py > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
for st in current new; do
  timeout -k 10 240 python -u tools/xcd_balance.py --sizes 1000000000 --rounds 3 --launches 30 --skews 0,20,-20 \
      --stream $st --json $O/xcd_$st.jsonl > $O/xcd_$st.txt 2>&1
  rc=$?; echo "xcd $st rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
done
one() {  # one <tag> <binary> <skew> <args...>
  local tag=$1 bin=$2; export MIREDUCE_XCD_SKEW=$3; shift 3
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
  done
  one "f64_cur_s20_$r" ./build/bin/reduction 20 --method=SUM --type=double --n=1e9
  one "f64_cur_sm20_$r" ./build/bin/reduction -20 --method=SUM --type=double --n=1e9
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
O = sys.argv[1]
for st in ("current", "new"):
    acc = collections.defaultdict(list); rot = set()
    for l in open(f"{O}/xcd_{st}.jsonl"):
        d = json.loads(l); acc[d["skew"]].append(d["us_per_launch"]); rot.add(json.dumps(d["xcc_rotation"]))
    for k, v in sorted(acc.items()):
        print(f"xcd stream={st:7s} skew {k:4d} us {sorted(v)}")
    print(f"xcd stream={st:7s} xcc rotations seen: {sorted(rot)}")
acc = collections.defaultdict(list)
for f in sorted(glob.glob(O + "/*_[123].jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[os.path.basename(f)[:-6].rsplit("_", 1)[0]].append((d["avg_ms"] * 1e3, d["gb_per_s"], d["verified"]))
for tag, v in sorted(acc.items()):
    print(f"{tag:14s} us {' '.join('%.2f' % x[0] for x in sorted(v)):32s} best GB/s {max(x[1] for x in v):8.1f} verified {all(x[2] for x in v)}")
PY
cat $O/summary.txt
