#!/bin/bash
# Round 6, final tree: the default GPU tier (timed), smoke(), the driver's default bench command, and
# one PMC pass (TCC) of the 8 GB headline kernel through the reduction app.
O=gpurun_out/r6_final
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  local t0=$SECONDS
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc wall=$((SECONDS - t0))s" | tee -a $O/status.txt
  case $rc in 0) ;; 1) [ "$name" = pytest ] || { echo "stopping after $name"; exit 1; } ;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=30 -p no:cacheprovider
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 --extras-file $O/bench_extras.json
R="./build/bin/reduction --method=SUM --type=double --n=1000000000 --fill=device --iterations=5 --log=none --master-log=none"
step tcc 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum \
    --output-format csv -d $O/tcc -o run -- $R
python3 tools/prof_summary.py $O/tcc $O/tcc > $O/tcc_summary.txt 2>&1
find $O/tcc -name "*counter_collection.csv" -exec cp {} $O/tcc_counters.csv \; ; rm -rf $O/tcc
cat $O/status.txt; tail -1 $O/pytest.out; head -c 400 $O/bench.out; echo; grep -h reduce_stream $O/tcc_summary.txt | head -3
