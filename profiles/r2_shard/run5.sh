#!/bin/bash
# After the auto graph chunk (one graph for kernel-only steps): fused/xrank GPU tests, then the
# headline at the 1 GB shard and at the default 8 GB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2_shard5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_xrank_gpu.py > $O/xrank_tests.log 2>&1 || { tail -30 $O/xrank_tests.log; exit 1; }
tail -1 $O/xrank_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --elements 125000000 --steps 1000 --warmup 20 --no-vector-extras > $O/bench_1gb_$i.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2>$O/bench_default.err || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r2_shard5/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("serial_gbps"), d["config"].get("collective"), d["config"].get("launch"), json.dumps(d.get("collective_tuning")))
PY
