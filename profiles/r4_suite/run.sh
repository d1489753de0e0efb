#!/bin/bash
# Round 4: the full GPU suite, smoke(), the default bench, and the 1 GB shard (the N=8 per-GPU work)
# through bench.py plain and under rocprofv3 --kernel-trace --stats (300 serial graph-replayed steps).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${PASS:-r4_suite}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py --elements 125000000 --steps 300 --warmup 20 --no-vector-extras > $O/shard.json 2> $O/shard.err
rc=$?; echo "shard rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --elements 125000000 --steps 300 \
    --warmup 20 --no-vector-extras > $O/shard_prof.json 2> $O/shard_prof.err
rc=$?; echo "prof rc=$rc" >> $O/status.txt
python3 tools/prof_db.py $O/prof/run_results.db --steady reduce_stream > $O/kernel_stats.txt 2>&1
rm -rf $O/prof
timeout -k 10 240 python -u tools/xcd_balance.py --sizes 125000000,1000000000 --rounds 5 --json $O/xcd_balance.jsonl > $O/xcd_balance.txt 2>&1
echo "xcd rc=$?" >> $O/status.txt
