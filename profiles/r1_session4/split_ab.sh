#!/usr/bin/env bash
# A/B of the streaming body's work split (MIREDUCE_SPLIT=stride|contig): correctness of the
# kernel suite under contig, then alternating runs of bench.py and the reduction app.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/split_ab; mkdir -p $O
export TMPDIR=/tmp
MIREDUCE_SPLIT=contig timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > $O/pytest_contig.txt 2>&1 || { tail -30 $O/pytest_contig.txt; exit 1; }
tail -2 $O/pytest_contig.txt
for rep in 1 2 3; do
  for S in stride contig; do
    MIREDUCE_SPLIT=$S timeout -k 10 120 python bench.py --steps 50 --warmup 10 2>/dev/null | grep '^{' > $O/b8g_${S}_$rep.json || exit 1
    MIREDUCE_SPLIT=$S timeout -k 10 120 python bench.py --elements 125000000 --steps 400 --warmup 20 2>/dev/null | grep '^{' > $O/b1g_${S}_$rep.json || exit 1
    for T in float int64; do
      MIREDUCE_SPLIT=$S timeout -k 10 120 build/bin/reduction --method=SUM --type=$T --n=1000000000 --iterations=50 --fill=device --noverify --log=none --master-log=none > $O/app_${T}_${S}_$rep.txt 2>&1 || exit 1
    done
    echo "rep $rep $S done"
  done
done
python - <<'PY'
import glob, json, re, statistics as st
O = "gpurun_out/split_ab"
for S in ("stride", "contig"):
    for tag in ("b8g", "b1g"):
        v = [json.load(open(f))["value"] for f in sorted(glob.glob(f"{O}/{tag}_{S}_*.json"))]
        print(f"{S:6s} {tag} bench GB/s: {v} median {st.median(v):.1f}")
    for T in ("float", "int64"):
        v = [float(re.search(r"Throughput = ([0-9.]+)", open(f).read()).group(1)) for f in sorted(glob.glob(f"{O}/app_{T}_{S}_*.txt"))]
        print(f"{S:6s} app {T} GB/s: {v} median {st.median(v):.1f}")
PY
