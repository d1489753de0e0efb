#!/bin/bash
# Round 3, GPU pass J: the whole GPU suite (bootstrap-port fix), the fp32 window sweep at the sizes
# pass I did not cover (1 GB, 4 GB), and a kernel trace of 300 serial 1 GB-shard steps.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
for n in 2.5e8 1e9; do
  timeout -k 10 300 ./build/bin/window_ab --type=float --n=$n --rounds=7 --iters=20 > $O/window_ab_f32_$n.txt 2>&1
  rc=$?; echo "window_ab_f32_$n rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --elements 125000000 \
    --steps 300 --warmup 10 --no-vector-extras --no-candidates > $O/bench_shard.json 2> $O/bench_shard.err
rc=$?; echo "prof_shard rc=$rc" >> $O/status.txt
python3 tools/prof_db.py $O/prof/run_results.db > $O/prof_stats.txt 2>&1
python3 tools/ab_kernels.py $O/prof/run_results.db > $O/prof_solo.md 2>&1
rm -rf $O/prof
exit $rc
