#!/bin/bash
# Balanced leftover (default) vs whole leftover tiles (MIREDUCE_BALANCE=0), per plan and size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_small3
mkdir -p $O
run() {  # tag n extra...
  local tag=$1 n=$2; shift 2
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/$tag -o t -- ./build/bin/reduction --method=SUM --type=double --n=$n --iterations=60 --timing=batch --log=none --fill=device "$@" > $O/$tag.log 2>&1 &&
  python tools/prof_db.py $O/$tag/t_results.db --csv $O/$tag.csv > /dev/null && rm -rf $O/$tag
}
for bal in 1 0; do
  export MIREDUCE_BALANCE=$bal
  for n in 16777216 125000000 250000000 500000000; do
    run b${bal}_def_$n $n || exit 1
    run b${bal}_512x16_$n $n --threads=512 --unroll=16 --wg-per-cu=1 || exit 1
    run b${bal}_512x8_$n $n --threads=512 --unroll=8 --wg-per-cu=1 || exit 1
    run b${bal}_256x4x2_$n $n --threads=256 --unroll=4 --wg-per-cu=2 || exit 1
  done
done
echo done
