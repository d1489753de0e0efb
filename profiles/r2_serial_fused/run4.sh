#!/bin/bash
# Serial candidates verified after all measurements (not between them): the two configs whose
# serial number fell ~6 % (2 GB f64, 8 GB bf16) and the headline, then the bench GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_serial4
mkdir -p $O
for c in gpu_256m_double_sum gpu_4g_bf16_sum xgmi_1b_double_sum; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 10 --no-vector-extras > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$c.json'));print('$c', d['value'], d.get('serial_gbps'), d.get('serial_candidates_gbps'), d['verified'])"
done
timeout -k 10 1000 python -u -m pytest tests/test_xrank_gpu.py tests/test_apps_gpu.py tests/test_fault_injection.py -m gpu -k "bench" -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
