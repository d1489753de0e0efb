#!/bin/bash
# Round 4, XCD skew pass 3: the element types whose default skew is 0 (bf16 window 4, int32 SUM
# window 2) with both signs, and the updated plan-tuning test.
set -o pipefail
O=${O:-gpurun_out/r4_xcd3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_xrank_gpu.py::test_bench_plan_tuning_at_the_eight_gpu_shard > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -le 1 ] || exit $rc
run() {  # run <tag> <skew> <config> <elements> <steps>
  MIREDUCE_XCD_SKEW=$2 timeout -k 10 180 python -u bench.py --config $3 --elements $4 --steps $5 --warmup 10 \
      --no-vector-extras --no-candidates --no-decompose --no-plan-tune > $O/$1.json 2> $O/$1.err
  local rc=$?; echo "$1 rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || { tail -5 $O/$1.err; exit $rc; }
}
for r in 1 2 3; do
  for sk in -20 0 20; do
    run "bf16_8g_s${sk}_$r" $sk gpu_4g_bf16_sum 4000000000 60
    MIREDUCE_XCD_SKEW=$sk timeout -k 10 120 ./build/bin/reduction --method=SUM --type=int --n=2e9 --fill=device \
        --iterations=60 --timing=batch --log=none --master-log=none --json=$O/i32sum_8g_s${sk}_$r.jsonl > $O/i32_${sk}_$r.out 2>&1
    rc=$?; echo "i32 $sk $r rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(O + "/*_s*_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    tag = os.path.basename(f)[:-5].rsplit("_", 1)[0]
    kp = d["config"]["kernel_plan"]
    acc[tag].append((d["ms_per_step"] * 1e3, d["value"], d["verified"], kp.get("xskew"), kp.get("window"), kp.get("grid")))
for f in sorted(glob.glob(O + "/i32sum_*.jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    tag = os.path.basename(f)[:-6].rsplit("_", 1)[0]
    acc[tag].append((d["avg_ms"] * 1e3, d["gb_per_s"], d["verified"], -999, d["window"], d["grid"]))
for tag, v in sorted(acc.items()):
    us = sorted(x[0] for x in v)
    print(f"{tag:18s} xskew {v[0][3]:4d} window {v[0][4]} grid {v[0][5]} us/step {' '.join('%.2f' % u for u in us):32s} best GB/s {max(x[1] for x in v):9.1f} verified {all(x[2] for x in v)}")
PY
cat $O/summary.txt; tail -2 $O/pytest.txt
