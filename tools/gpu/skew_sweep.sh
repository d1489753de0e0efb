#!/bin/bash
# XCD-weighted split sweep with the reduction app: for each plan in $PLANS (";"-separated app
# argument lists) and each skew in $SKEWS (permille, MIREDUCE_XCD_SKEW), one process per point,
# kernel-only batch timing, $ROUNDS interleaved rounds; summary: us per reduction per (plan, skew).
#   O=gpurun_out/skew ROUNDS=2 SKEWS="0 20" PLANS="--method=SUM --type=double --n=1e9" bash tools/gpu/skew_sweep.sh
set -o pipefail
O=${O:-gpurun_out/skew_sweep}
ROUNDS=${ROUNDS:-2}
SKEWS=${SKEWS:-"0 10 20 30"}
PLANS=${PLANS:-"--method=SUM --type=double --n=1e9;--method=SUM --type=float --n=2e9;--method=SUM --type=bf16 --n=4e9"}
mkdir -p $O
IFS=';' read -r -a plans <<< "$PLANS"
for r in $(seq 1 $ROUNDS); do
  for i in "${!plans[@]}"; do
    for sk in $SKEWS; do
      tag="p${i}_s${sk}_$r"
      MIREDUCE_XCD_SKEW=$sk timeout -k 10 120 ./build/bin/reduction ${plans[$i]} --fill=device --iterations=60 \
          --timing=batch --log=none --master-log=none --json=$O/$tag.jsonl > $O/$tag.out 2>&1
      rc=$?; echo "$tag rc=$rc" >> $O/status.txt
      [ $rc -eq 0 ] || { tail -3 $O/$tag.out; exit $rc; }
    done
  done
done
python3 - "$O" "$PLANS" <<'PY' > $O/summary.txt
import collections, glob, json, os, sys
plans = sys.argv[2].split(";")
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/p*_s*_*.jsonl")):
    p, s, _ = os.path.basename(f)[:-6].split("_")
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[(int(p[1:]), int(s[1:]))].append((d["avg_ms"] * 1e3, d["verified"]))
for (p, s), v in sorted(acc.items()):
    print(f"{plans[p]:45s} skew {s:4d} us {' '.join('%.2f' % x[0] for x in sorted(v)):24s} verified {all(x[1] for x in v)}")
PY
cat $O/summary.txt
