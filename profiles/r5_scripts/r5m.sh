#!/bin/bash
# Round 5: the HBM-filling gap's counters, one launch vs segmented (r3_hbmfill saw +35 % DRAM-credit
# stalls per request at 292 GB): reduction app, fp32 SUM of 7.3e10 floats, segment_bytes -1 (one
# launch) vs 0 (auto: 8 GiB launches). Timing first (2 rounds, batch), then one PMC pass each.
set -o pipefail
O=gpurun_out/r5m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B=./build/bin/reduction
for r in 1 2; do
  for seg in -1 0; do
    timeout -k 10 240 $B --method=SUM --type=float --n=73e9 --fill=device --pattern=iotamod --iterations=3 \
        --timing=batch --segment-bytes=$seg --log=none --master-log=none --json=$O/time_seg${seg}.jsonl > $O/time_seg${seg}_$r.out 2>&1
    rc=$?; echo "time seg$seg r$r rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -3 $O/time_seg${seg}_$r.out; exit $rc; }
  done
done
P2=TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum,TCC_TAG_STALL_sum,TCC_HIT_sum
for seg in -1 0; do
  timeout -s KILL 240 rocprofv3 --pmc $P2 --output-format csv -d $O/pmc_seg$seg -o run -- $B --method=SUM --type=float \
      --n=73e9 --fill=device --pattern=iotamod --iterations=2 --segment-bytes=$seg --log=none --master-log=none > $O/pmc_seg$seg.out 2>&1
  rc=$?; echo "pmc seg$seg rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -3 $O/pmc_seg$seg.out; exit $rc; }
done
python3 - "$O" <<'PY' > $O/summary.txt
import csv, glob, json, os, sys, collections
O = sys.argv[1]
for seg in ("-1", "0"):
    rows = [json.loads(l) for l in open(f"{O}/time_seg{seg}.jsonl") if l.strip()]
    print(f"segment_bytes {seg:>2}: GB/s " + " ".join("%.1f" % r["gb_per_s"] for r in rows) +
          f"  segments {rows[0].get('segments')}  verified {all(r.get('verified') for r in rows)}")
for seg in ("-1", "0"):
    f = (glob.glob(f"{O}/pmc_seg{seg}/**/*counter_collection.csv", recursive=True) or [None])[0]
    if f is None:
        print(f"seg {seg}: no counter file"); continue
    tot = collections.defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f)):
        if "reduce_stream" not in r.get("Kernel_Name", ""):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r.get("Dispatch_Id"))
    req = tot.get("TCC_EA0_RDREQ_sum", 0) or 1
    print(f"seg {seg:>2}: {len(disp)} dispatches; " + ", ".join(f"{k} {v:.4g}" for k, v in sorted(tot.items())) +
          f"; DRAM-credit stalls per request {tot.get('TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum', 0) / req:.3f}")
PY
cat $O/summary.txt
find $O -name "*.db" -delete
