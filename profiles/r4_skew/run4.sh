#!/bin/bash
# Round 4: the 16-bit SUM body with its packed adds written out (build/ab_pair: two unroll slots
# per step, one v_pk_add_f32 per element) vs as shipped (build/ab_head: hipcc's SLP pairing, whose
# schedule differs between the skewed path's loop copies). bf16 SUM at skew 0 / 10 / 20, f16 SUM
# at 0; same box, interleaved, 3 rounds, 8 GB per reduction.
set -o pipefail
O=${O:-gpurun_out/r4_skew4}
mkdir -p $O
one() {  # one <tag> <binary> <skew> <args...>
  local tag=$1 bin=$2; export MIREDUCE_XCD_SKEW=$3; shift 3
  timeout -k 10 120 $bin "$@" --fill=device --iterations=60 --timing=batch --log=none \
      --master-log=none --json=$O/$tag.jsonl > $O/$tag.out 2>&1
  local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -3 $O/$tag.out; exit $rc; }
}
for r in 1 2 3; do
  for v in head pair; do
    B=./build/ab_$v/reduction
    for sk in 0 10 20; do one "bf16_${v}_s${sk}_$r" $B $sk --method=SUM --type=bf16 --n=4e9; done
    one "f16_${v}_s0_$r" $B 0 --method=SUM --type=half --n=4e9
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[os.path.basename(f)[:-6].rsplit("_", 1)[0]].append((d["avg_ms"] * 1e3, d["gb_per_s"], d["verified"]))
for tag, v in sorted(acc.items()):
    print(f"{tag:16s} us {' '.join('%.2f' % x[0] for x in sorted(v)):28s} best GB/s {max(x[1] for x in v):8.1f} verified {all(x[2] for x in v)}")
PY
cat $O/summary.txt
