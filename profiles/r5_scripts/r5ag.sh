#!/bin/bash
# Round 5, final tree: rocprofv3 kernel stats of the default bench, and one PMC pass (TCC) of the
# 8 GB headline kernel through the reduction app.
O=gpurun_out/r5ag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -s KILL $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  case $rc in 0|1) ;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
step kt 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 bench.py --no-vector-extras --steps 20 --warmup 5 \
    --extras-file $O/kt_extras.json
R="./build/bin/reduction --method=SUM --type=double --n=1000000000 --fill=device --iterations=5 --log=none --master-log=none"
step tcc 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum \
    --output-format csv -d $O/tcc -o run -- $R
python3 tools/prof_summary.py $O/tcc $O/tcc > $O/tcc_summary.txt 2>&1
find $O/tcc -name "*counter_collection.csv" -exec cp {} $O/tcc_counters.csv \; ; rm -rf $O/tcc
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/kt -name "*.db" -exec python3 tools/prof_db.py {} \; > $O/kt_prof_db.txt 2>&1
rm -rf $O/kt
cat $O/status.txt; head -5 $O/kernel_stats.csv; grep -h reduce_stream $O/tcc_summary.txt | head -3
