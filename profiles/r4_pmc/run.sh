#!/bin/bash
# Round 4: PMC counters of the 8 GB headline kernel (window-4 plan, anchored XCD-weighted split) at
# skew 0 and at the default 20, two passes of their own per skew (TCC: HBM read requests / hits;
# SQ: wave cycles, busy, waits, VALU, VMEM reads). The anchor adds one 8-byte load per workgroup.
O=gpurun_out/r4_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -s KILL $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  case $rc in 0|1) ;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
B=./build/bin/reduction
R="$B --method=SUM --type=double --n=1000000000 --fill=device --iterations=5 --log=none --master-log=none"
for sk in 0 20; do
  export MIREDUCE_XCD_SKEW=$sk
  step tcc_s$sk 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum \
      --output-format csv -d $O/tcc_s$sk -o run -- $R
  step sq_s$sk 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
      SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq_s$sk -o run -- $R
done
for d in tcc_s0 sq_s0 tcc_s20 sq_s20; do
  python3 tools/prof_summary.py $O/$d $O/$d > $O/${d}_summary.txt 2>&1
  find $O/$d -name "*counter_collection.csv" -exec cp {} $O/${d}_counters.csv \; ; rm -rf $O/$d
done
grep -h "reduce_stream" $O/*_summary.txt > $O/summary.txt; cat $O/summary.txt
