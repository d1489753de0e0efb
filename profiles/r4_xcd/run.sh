#!/bin/bash
# Round 4: XCD-weighted split of the window body (MIREDUCE_XCD_SKEW = permille of the rounds given
# extra to the odd workgroups). Correctness first, then the production kernel's per-XCD end
# stamps and the headline protocol at the 1 GB shard and at 8 GB, skews interleaved over rounds.
set -o pipefail
O=${O:-gpurun_out/r4_xcd}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py::test_xcd_weighted_split \
  tests/test_apps_gpu.py::test_bench_graph_capture_failure_falls_back_on_all_ranks \
  tests/test_kernels_gpu.py::test_every_variant > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -5 $O/pytest.txt; exit $rc; }
for sk in 0 16; do
  MIREDUCE_XCD_SKEW=$sk timeout -k 10 200 python -u tools/xcd_balance.py --sizes 125000000,1000000000 --rounds 3 \
      > $O/xcd_skew$sk.txt 2>&1
  rc=$?; echo "xcd $sk rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
done
run() {  # run <tag> <skew> <elements> <steps>
  MIREDUCE_XCD_SKEW=$2 timeout -k 10 180 python -u bench.py --elements $3 --steps $4 --warmup 10 --no-vector-extras \
      --no-candidates --no-decompose --no-plan-tune > $O/$1.json 2> $O/$1.err
  local rc=$?; echo "$1 rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || { tail -5 $O/$1.err; exit $rc; }
}
for r in 1 2 3; do
  for sk in 0 8 16 24; do
    run "g1_s${sk}_$r" $sk 125000000 400
    run "g8_s${sk}_$r" $sk 1000000000 60
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(O + "/g*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    tag = os.path.basename(f)[:-5].rsplit("_", 1)[0]
    acc[tag].append((d["ms_per_step"] * 1e3, d["value"], d["verified"], d["config"]["kernel_plan"].get("xskew")))
for tag, v in sorted(acc.items()):
    us = sorted(x[0] for x in v)
    print(f"{tag:10s} xskew {v[0][3]:4d} us/step {' '.join('%.2f' % u for u in us):32s} best GB/s {max(x[1] for x in v):9.1f} verified {all(x[2] for x in v)}")
PY
cat $O/summary.txt
