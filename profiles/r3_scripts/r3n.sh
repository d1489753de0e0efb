#!/bin/bash
# Round 3, GPU pass N: (1) rocprofv3 kernel trace of 300 graph-replayed one-lane fused steps at the
# N=8 shard (125M doubles = 1 GB), period = kernel + gap (VERDICT r2 item 5's evidence);
# (2) PMC counters of the 8 GB headline kernel (window-4 plan) in two passes of their own.
O=gpurun_out/r3n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  case $rc in 0|1) ;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
step shard_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard -o run -- python3 bench.py \
    --elements 125000000 --steps 300 --warmup 10 --no-vector-extras --no-candidates --no-plan-tune
python3 tools/kernel_gaps.py $O/shard --match "reduce_stream" --bytes 1e9 --skip 13 > $O/shard_gaps.txt 2>&1
find $O/shard -name "*kernel_stats.csv" -exec cp {} $O/shard_kernel_stats.csv \;
rm -rf $O/shard
B=./build/bin/reduction
R="$B --method=SUM --type=double --n=1000000000 --fill=device --iterations=5 --log=none --master-log=none"
step pmc_tcc 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum \
    GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_tcc -o run -- $R
step pmc_sq 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -o run -- $R
python3 tools/prof_summary.py $O/pmc_tcc $O/pmc_tcc > $O/pmc_tcc_summary.txt 2>&1
python3 tools/prof_summary.py $O/pmc_sq $O/pmc_sq > $O/pmc_sq_summary.txt 2>&1
for d in pmc_tcc pmc_sq; do find $O/$d -name "*counter_collection.csv" -exec cp {} $O/${d}_counters.csv \; ; rm -rf $O/$d; done
exit 0
