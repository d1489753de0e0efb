#!/bin/bash
# The N=8 per-GPU shard (125M doubles = 1 GB) and the reference default (2^24 doubles = 128 MiB):
# kernel-only time warm / cold (rocprofv3), and bench.py at the 1 GB shard with every cross-rank
# combine candidate (collective_tuning) on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_shard
mkdir -p $O
for n in 16777216 125000000; do
  for t in warm cold; do
    extra="--timing=batch"; [ $t = cold ] && extra="--cold"
    timeout -k 10 120 rocprofv3 --kernel-trace -d $O/${t}_$n -o t -- ./build/bin/reduction --method=SUM --type=double --n=$n --iterations=60 $extra --log=none --fill=device > $O/${t}_$n.log 2>&1 || exit 1
    db=$(ls $O/${t}_$n/*/t_results.db $O/${t}_$n/t_results.db 2>/dev/null | head -1)
    python tools/prof_db.py "$db" > $O/${t}_$n.txt && rm -rf $O/${t}_$n
  done
done
timeout -k 10 300 python bench.py --elements 125000000 --steps 400 --warmup 40 --no-vector-extras > $O/bench_1gb.json 2>$O/bench_1gb.err || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-vector-extras > $O/bench_default.json 2>$O/bench_default.err || exit 1
cat $O/*.txt
python - <<'PY'
import json
for f in ("gpurun_out/r2_shard/bench_1gb.json", "gpurun_out/r2_shard/bench_default.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("serial_gbps"), d.get("collective"), json.dumps(d.get("collective_tuning")))
PY
