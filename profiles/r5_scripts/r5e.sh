#!/bin/bash
# Round 5: segmented launches for the HBM-filling config (library segmentation, 4/8/16 GiB vs one
# launch), the launch floor, the GPU suite, then the N=1 bench and the HBM-fill bench config.
set -o pipefail
O=gpurun_out/r5e
mkdir -p $O
st() { echo "$1 rc=$2" | tee -a $O/status.txt; }
timeout -k 10 180 ./build/bin/launch_floor --rounds=7 --launches=200 > $O/launch_floor.txt 2>&1
rc=$?; st launch_floor $rc; cat $O/launch_floor.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 tools/hbm_chunks.py --fraction 0.9 --rounds 3 --segments 4,8,16 --json $O/hbm_segments.jsonl > $O/hbm_segments.txt 2>&1
rc=$?; st hbm_segments $rc; grep "^\[hbm\]" $O/hbm_segments.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; st pytest $rc; tail -4 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --extras-file $O/bench_extras_n1.json > $O/bench.json 2> $O/bench.err
rc=$?; st bench $rc; cat $O/bench.json; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 bench.py --config hbm_fill_fp32_sum --steps 5 --warmup 1 --no-vector-extras --extras-file $O/bench_extras_hbm.json > $O/bench_hbm.json 2> $O/bench_hbm.err
rc=$?; st bench_hbm $rc; cat $O/bench_hbm.json
exit $rc
