#!/bin/bash
# Round 4: the 1 GB shard (the N=8 per-GPU work, 125M doubles) with the round-4 kernel (finisher-only
# channel loads, XCD-weighted split), 300 serial graph-replayed fused steps: bench.py's clock, then
# the same command under rocprofv3 --kernel-trace --stats (kernel period from the trace). Then the
# XCD skew for the other window element types (fp32 SUM 8 GB, int32 SUM 8 GB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/r4_shard}
mkdir -p $O
timeout -k 10 300 python -u bench.py --elements 125000000 --steps 300 --warmup 20 --no-vector-extras > $O/shard.json 2> $O/shard.err
rc=$?; echo "shard rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --elements 125000000 --steps 300 \
    --warmup 20 --no-vector-extras --no-decompose --no-candidates > $O/shard_prof.json 2> $O/shard_prof.err
rc=$?; echo "prof rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_db.py $O/prof/run_results.db --steady reduce_stream > $O/kernel_stats.txt 2>&1
rm -rf $O/prof
run() {  # run <tag> <skew> <config> <elements> <steps>
  MIREDUCE_XCD_SKEW=$2 timeout -k 10 180 python -u bench.py --config $3 --elements $4 --steps $5 --warmup 10 \
      --no-vector-extras --no-candidates --no-decompose --no-plan-tune > $O/$1.json 2> $O/$1.err
  local rc=$?; echo "$1 rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || { tail -5 $O/$1.err; exit $rc; }
}
for r in 1 2 3; do
  for sk in 0 20 -20; do
    run "f32_8g_s${sk}_$r" $sk hbm_fill_fp32_sum 2000000000 60
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(O + "/*_s*_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    tag = os.path.basename(f)[:-5].rsplit("_", 1)[0]
    acc[tag].append((d["ms_per_step"] * 1e3, d["value"], d["verified"], d["config"]["kernel_plan"].get("xskew"),
                     d["config"]["kernel_plan"].get("window")))
for tag, v in sorted(acc.items()):
    us = sorted(x[0] for x in v)
    print(f"{tag:16s} xskew {v[0][3]:4d} window {v[0][4]} us/step {' '.join('%.2f' % u for u in us):32s} best GB/s {max(x[1] for x in v):9.1f} verified {all(x[2] for x in v)}")
for f in ("shard.json", "shard_prof.json"):
    d = json.loads(open(O + "/" + f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["verified"], d.get("plan_tuning"))
PY
cat $O/summary.txt $O/kernel_stats.txt
