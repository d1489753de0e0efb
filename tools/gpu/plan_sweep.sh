#!/bin/bash
# Launch-plan sweep with the reduction app at one size: each plan in $PLANS (";"-separated app
# argument lists, e.g. "--threads=256 --unroll=4 --wg-per-cu=3 --window=0") x each timing in
# $TIMINGS (batch = back-to-back launches, per-iter = the reference's one timed launch at a time),
# $ROUNDS interleaved rounds, one process per point, verified. Summary: median us per reduction.
#   O=gpurun_out/small N=16777216 PLANS="...;..." bash tools/gpu/plan_sweep.sh
set -o pipefail
O=${O:-gpurun_out/plan_sweep}
N=${N:-16777216}
TYPE=${TYPE:-double}
METHOD=${METHOD:-SUM}
ITERS=${ITERS:-100}
ROUNDS=${ROUNDS:-2}
TIMINGS=${TIMINGS:-"batch per-iter"}
PLANS=${PLANS:-"--threads=256 --unroll=4 --wg-per-cu=3 --window=0"}
mkdir -p $O
IFS=';' read -r -a plans <<< "$PLANS"
printf '%s\n' "${plans[@]}" > $O/plans.txt
for r in $(seq 1 $ROUNDS); do
  for i in "${!plans[@]}"; do
    for tm in $TIMINGS; do
      tag="p${i}_${tm}_$r"
      timeout -k 10 120 ./build/bin/reduction --method=$METHOD --type=$TYPE --n=$N ${plans[$i]} --fill=device \
          --iterations=$ITERS --timing=$tm --log=none --master-log=none --json=$O/$tag.jsonl > $O/$tag.out 2>&1
      rc=$?; echo "$tag rc=$rc" >> $O/status.txt
      [ $rc -eq 0 ] || { tail -3 $O/$tag.out; exit $rc; }
    done
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import collections, glob, json, os, sys
plans = open(sys.argv[1] + "/plans.txt").read().splitlines()
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/p*_*_*.jsonl")):
    p, tm, _ = os.path.basename(f)[:-6].split("_")
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[(int(p[1:]), tm)].append((d["median_ms"] * 1e3, d["verified"], d.get("grid"), d.get("window")))
for (p, tm), v in sorted(acc.items()):
    print(f"{plans[p]:60s} {tm:8s} median us {' '.join('%.2f' % x[0] for x in v):20s} "
          f"grid {v[0][2]} window {v[0][3]} verified {all(x[1] for x in v)}")
PY
cat $O/summary.txt
