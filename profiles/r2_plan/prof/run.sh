#!/bin/bash
# The new 8 GB plan (256x8x1) under rocprofv3: kernel stats, then HBM read requests (PMC, own run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_plan_prof
mkdir -p $O
A="./build/bin/reduction --method=SUM --type=double --n=1000000000 --iterations=20 --log=none"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/stats -o k --output-format csv -- $A > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d $O/pmc -o p --output-format csv -- $A > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
grep -h "reduce_stream" $(find $O/stats -name "*kernel_stats.csv") | cut -c1-250
