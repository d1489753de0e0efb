#!/bin/bash
# Every BASELINE.json GPU config through bench.py on one GPU (current tree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${O:-gpurun_out/configs}
mkdir -p $O; export O
for c in gpu_256m_double_sum gpu_256m_int64_min xgmi_1b_double_sum gpu_4g_bf16_sum xgmi_1b_double_norm2 xgmi_1b_double_maxloc; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 10 --no-vector-extras --extras-file $O/$c.extras.json \
      > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
done
timeout -k 10 600 python bench.py --config hbm_fill_fp32_sum --steps 5 --warmup 1 --extras-file $O/hbm_fill_fp32_sum.extras.json \
    > $O/hbm_fill_fp32_sum.json 2> $O/hbm_fill_fp32_sum.err || { tail -5 $O/hbm_fill_fp32_sum.err; exit 1; }
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob(os.environ.get("O", "gpurun_out/configs") + "/*.json")):
    if f.endswith(".extras.json"):
        continue
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["unit"], d["ms_per_step"], d.get("verified"), d["config"].get("collective"),
          (d.get("summary") or {}).get("plans"))
PY
