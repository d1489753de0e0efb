#!/bin/bash
# Round 5 (r5f rerun): the bench GPU tests (test_xrank_gpu.py: the rest of the suite passed in r5f),
# the launch floor with the coarse-slot A/B, the N=1 bench, the HBM-filling bench config
# (segmented by default now), and a kernel trace of both under rocprofv3.
set -o pipefail
O=gpurun_out/r5h
mkdir -p $O
st() { echo "$1 rc=$2" | tee -a $O/status.txt; }
true

timeout -k 10 1000 python3 -u -m pytest tests/test_xrank_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; st pytest $rc; tail -4 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --extras-file $O/bench_extras_n1.json > $O/bench.json 2> $O/bench.err
rc=$?; st bench $rc; cat $O/bench.json; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 bench.py --config hbm_fill_fp32_sum --steps 5 --warmup 1 --no-vector-extras --extras-file $O/bench_extras_hbm.json > $O/bench_hbm.json 2> $O/bench_hbm.err
rc=$?; st bench_hbm $rc; cat $O/bench_hbm.json; [ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run -- python3 bench.py --steps 20 --warmup 5 --no-vector-extras --extras-file $O/prof_bench_extras.json > $O/prof_bench.json 2> $O/prof_bench.err
rc=$?; st prof_bench $rc; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_hbm -o run -- python3 bench.py --config hbm_fill_fp32_sum --steps 3 --warmup 1 --no-vector-extras --no-candidates --extras-file $O/prof_hbm_extras.json > $O/prof_hbm.json 2> $O/prof_hbm.err
rc=$?; st prof_hbm $rc
for d in prof_bench prof_hbm; do
  db=$(ls $O/$d/*/run_results.db $O/$d/run_results.db 2>/dev/null | head -1)
  [ -n "$db" ] && python3 tools/prof_db.py "$db" > $O/$d.stats.txt 2>&1
  f=$(ls $O/$d/*/run_kernel_stats.csv $O/$d/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] && cp "$f" $O/$d.kernel_stats.csv
  rm -rf $O/$d
done
exit $rc
