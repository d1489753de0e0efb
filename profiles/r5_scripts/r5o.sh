#!/bin/bash
# Round 5: after equal-size segments — the segmented / fan-in GPU tests and the HBM-filling bench.
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
st() { echo "$1 rc=$2" | tee -a $O/status.txt; }
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fanin_gpu.py -m gpu -x -q -k "segment or fanin or anchor" --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; st pytest $rc; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --config hbm_fill_fp32_sum --steps 5 --warmup 1 --no-vector-extras --extras-file $O/bench_hbm_extras.json > $O/bench_hbm.json 2> $O/bench_hbm.err
rc=$?; st bench_hbm $rc; cat $O/bench_hbm.json
exit $rc
