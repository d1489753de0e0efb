#!/bin/bash
# Round 3, GPU pass H: window confirmation sweep, the whole GPU suite, the driver's bench + rocprof.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 1e9 1.25e8; do
  timeout -k 10 300 ./build/bin/window_ab --n=$n --rounds=7 --iters=20 > $O/window_ab_$n.txt 2>&1
  rc=$?; echo "window_ab_$n rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py --elements 125000000 --steps 300 --warmup 10 --no-vector-extras \
    > $O/bench_1gb_shard.json 2> $O/bench_1gb_shard.err
rc=$?; echo "bench_1gb rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
    --no-vector-extras > $O/bench_prof.json 2> $O/bench_prof.err
rc=$?; echo "prof rc=$rc" >> $O/status.txt
python3 tools/prof_db.py $O/prof/run_results.db > $O/prof_stats.txt 2>&1
python3 tools/ab_kernels.py $O/prof/run_results.db > $O/prof_solo.md 2>&1
rm -rf $O/prof
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt
tail -3 $O/pytest_gpu.log
