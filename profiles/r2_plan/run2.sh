#!/bin/bash
# After the sched_barrier between a tile's loads and its adds (all UNROLL loads in flight):
# streaming-kernel numerics, the same head-to-head as run.sh, then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_plan
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_ops.py tests/test_half.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests2.txt 2>&1 || { tail -30 $O/tests2.txt; exit 1; }
tail -1 $O/tests2.txt
timeout -k 10 400 python -u tools/tune.py --dtype float64 --op sum --ns 500000000,1000000000 --rounds 12 --iters 20 \
  --blocks 256,512 --unrolls 8,16 --wgs 1 --policies nt > $O/h2h_f64_2.txt 2>&1 || { tail -20 $O/h2h_f64_2.txt; exit 1; }
grep -v "^\[tune\]" $O/h2h_f64_2.txt
timeout -k 10 300 python -u tools/tune.py --dtype int64 --op max --ns 1000000000 --rounds 8 --iters 20 \
  --blocks 512 --unrolls 8,16 --wgs 1 --policies nt > $O/h2h_i64_2.txt 2>&1 || { tail -20 $O/h2h_i64_2.txt; exit 1; }
grep -v "^\[tune\]" $O/h2h_i64_2.txt
timeout -k 10 300 python bench.py > $O/bench_default2.json 2> $O/bench_default2.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_default2.json'));print(d['value'], d['config']['collective'], d.get('serial_gbps'), d.get('collective_tuning'))"
