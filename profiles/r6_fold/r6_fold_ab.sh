#!/bin/bash
# Round 6: the split fold for the widening sums (int32 SUM into int64, fp32 SUM into fp64) against the
# tree before it (abtmp/cur: HEAD's extension + libmireduce.so, same sources otherwise), same box.
# tools/op_ab.py in each tree, trees alternating, 3 rounds each; 1e9 elements (4 GB of 4-byte types);
# the tuned plan ("auto") and the window-4, one-workgroup-per-CU plan the int32 SUM default had to
# leave in round 3 (its chain of 4 dependent 64-bit adds per vector), fp64 SUM as the control.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r6_fold_ab
mkdir -p $out
V="auto;block=256,unroll=8,wg_per_cu=1,window=4;block=256,unroll=8,wg_per_cu=2,window=2"
for r in 1 2 3; do
  for side in old new; do
    if [ $side = old ]; then t=abtmp/cur/tools/op_ab.py; else t=tools/op_ab.py; fi
    timeout -k 10 300 python -u $t --n 1e9 --pairs int32:sum,float32:sum,float64:sum --variants "$V" --rounds 3 \
      > $out/${side}_$r.txt 2>&1 || exit $?
    echo "== $side $r"; grep "^|" $out/${side}_$r.txt | tail -n +3
  done
done
