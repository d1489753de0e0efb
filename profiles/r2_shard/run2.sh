#!/bin/bash
# bench.py at the N=8 shard (1 GB per GPU) and the default, with the adaptive tuning length.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2_shard
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread -p no:cacheprovider tests/test_xrank_gpu.py -k "tunes" > $O/tune_test.log 2>&1 || { tail -20 $O/tune_test.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --elements 125000000 --steps 400 --warmup 40 --no-vector-extras > $O/bench2_1gb_$i.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-vector-extras > $O/bench2_default.json 2>/dev/null || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r2_shard/bench2_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("serial_gbps"), d["config"].get("collective"), json.dumps(d.get("collective_tuning")))
PY
