#!/bin/bash
# Fixed-overhead study: kernel-only time (rocprofv3) and event-timed time per reduction vs size
# (float64 SUM, kernel 7), warm (batch) and cold (--cold: MALL/L2 evicted before each iteration).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_small
mkdir -p $O
for n in 1024 65536 1048576 4194304 16777216 125000000; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/p_$n -o t -- ./build/bin/reduction --method=SUM --type=double --n=$n --iterations=100 --timing=batch --log=none --json=$O/warm_$n.json > $O/warm_$n.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/c_$n -o t -- ./build/bin/reduction --method=SUM --type=double --n=$n --iterations=30 --cold --log=none --json=$O/cold_$n.json > $O/cold_$n.log 2>&1 || exit 1
done
echo done
