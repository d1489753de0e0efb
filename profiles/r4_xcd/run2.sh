#!/bin/bash
# Round 4, XCD skew pass 2: finer skews for f64 at 1 GB / 8 GB, the other window element types, and
# the default bench (now tuning skew 0 / 20 / 40 on the node).
set -o pipefail
O=${O:-gpurun_out/r4_xcd2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_fanin_gpu.py > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -5 $O/pytest.txt; exit $rc; }
run() {  # run <tag> <skew> <config> <elements> <steps>
  MIREDUCE_XCD_SKEW=$2 timeout -k 10 180 python -u bench.py --config $3 --elements $4 --steps $5 --warmup 10 \
      --no-vector-extras --no-candidates --no-decompose --no-plan-tune > $O/$1.json 2> $O/$1.err
  local rc=$?; echo "$1 rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || { tail -5 $O/$1.err; exit $rc; }
}
for r in 1 2 3; do
  for sk in 0 20 32 44; do
    run "f64_1g_s${sk}_$r" $sk xgmi_1b_double_sum 125000000 400
    run "f64_8g_s${sk}_$r" $sk xgmi_1b_double_sum 1000000000 60
  done
  for sk in 0 20; do
    run "bf16_8g_s${sk}_$r" $sk gpu_4g_bf16_sum 4000000000 60
    run "i64min_2g_s${sk}_$r" $sk gpu_256m_int64_min 268435456 200
  done
done
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo "bench rc=$?" >> $O/status.txt
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(O + "/*_s*_*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    tag = os.path.basename(f)[:-5].rsplit("_", 1)[0]
    acc[tag].append((d["ms_per_step"] * 1e3, d["value"], d["verified"], d["config"]["kernel_plan"].get("xskew")))
for tag, v in sorted(acc.items()):
    us = sorted(x[0] for x in v)
    print(f"{tag:16s} xskew {v[0][3]:4d} us/step {' '.join('%.2f' % u for u in us):32s} best GB/s {max(x[1] for x in v):9.1f} verified {all(x[2] for x in v)}")
d = json.loads(open(O + "/bench_default.json").read().strip().splitlines()[-1])
print("bench default", d["value"], d["ms_per_step"], d.get("plan_tuning"), d["config"]["kernel_plan"].get("xskew"))
PY
cat $O/summary.txt
