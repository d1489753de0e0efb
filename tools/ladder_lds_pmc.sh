#!/usr/bin/env bash
# LDS bank conflicts of the Harris ladder kernels k0..k6 (the whitepaper's point: interleaved
# addressing k1 conflicts, sequential addressing k2 does not) + the streaming kernel k7.
# One rocprofv3 --pmc run per kernel (counters only, no trace domains).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ladder_pmc
mkdir -p $O
for k in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES -d $O/k$k -o run --output-format csv -- \
    build/bin/reduction --method=SUM --type=int --n=16777216 --kernel=$k --iterations=3 --noverify --log=none --master-log=none > /dev/null
done
python3 - <<'PY'
import csv, glob, collections
print("kernel,dispatches,SQ_LDS_BANK_CONFLICT,SQ_INSTS_LDS,SQ_WAVES,conflicts_per_lds_inst")
for k in range(8):
    agg = collections.defaultdict(float); disp = set()
    for f in glob.glob(f"gpurun_out/ladder_pmc/k{k}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "fill" not in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
    n = max(len(disp), 1)
    c, i, w = agg["SQ_LDS_BANK_CONFLICT"] / n, agg["SQ_INSTS_LDS"] / n, agg["SQ_WAVES"] / n
    print(f"{k},{len(disp)},{c:.0f},{i:.0f},{w:.0f},{(c / i if i else 0):.3f}")
PY
