#!/bin/bash
# One SQ/GRBM counter pass of the headline kernel (1e9 doubles, 8 GB, the reduction app, 5 launches):
# waves, instruction mix per wave, busy cycles — the final tree's counterpart of r4_pmc.
O=gpurun_out/r6_sq; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="./build/bin/reduction --method=SUM --type=double --n=1000000000 --fill=device --iterations=5 --log=none --master-log=none"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $O/raw -o run -- $R > $O/app.txt 2>&1 || exit $?
python3 tools/prof_summary.py $O/raw $O/raw > $O/sq_summary.txt 2>&1
find $O/raw -name "*counter_collection.csv" -exec cp {} $O/sq_counters.csv \; ; rm -rf $O/raw
grep -h reduce_stream $O/sq_summary.txt | head -12
