#!/bin/bash
# why is the HBM-filling fp32 SUM (295 GB) ~3.5 % below the 8 GB configs?
#  1. GB/s vs array size (8 GB .. 292 GB), interleaved split (default) and contiguous split
#  2. PMC at 8 GB vs 292 GB: UTCL1 translation misses / stalls, UTCL2 busy, EA read requests & stalls
# Every GPU step has its own time limit; a timeout / crash ends the script.
O=${O:-gpurun_out/hbmfill}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B=./build/bin/reduction
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  case $rc in 0|1) ;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
for r in 1 2; do
  for n in 2000000000 20000000000 60000000000 73000000000; do
    step size_r${r}_$n 120 $B --method=SUM --type=float --n=$n --fill=device \
      --pattern=iotamod --iterations=10 --log=none --master-log=none --json=$O/size_stride.jsonl
  done
done
# (round 3: the contiguous split was 2-10 % slower than the interleaved one at every size; removed in round 6)
P1=TCP_UTCL1_TRANSLATION_MISS_sum,TCP_UTCL1_TRANSLATION_HIT_sum,TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum,TCP_UTCL1_STALL_MULTI_MISS_sum,GRBM_UTCL2_BUSY,GRBM_GUI_ACTIVE
P2=TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum,TCC_TAG_STALL_sum,TCC_HIT_sum
for n in 73000000000; do
  step pmc1_$n 120 rocprofv3 --pmc $P1 --output-format csv -d $O/pmc1_$n -o run -- $B --method=SUM --type=float \
      --n=$n --fill=device --pattern=iotamod --iterations=3 --log=none --master-log=none
  step pmc2_$n 120 rocprofv3 --pmc $P2 --output-format csv -d $O/pmc2_$n -o run -- $B --method=SUM --type=float \
      --n=$n --fill=device --pattern=iotamod --iterations=3 --log=none --master-log=none
done
