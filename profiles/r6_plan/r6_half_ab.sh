#!/bin/bash
# Round 6 follow-up of r6_plan_ab.sh: that run split the 16-bit compares by DTYPE (fp16 MIN ahead
# on the window-4 one-workgroup-per-CU plan at 2 / 4 GB, bf16 MAX behind on it). All four
# dtype x op pairs, three plans, 1 / 2 / 4 GB, 4 interleaved rounds (tools/op_ab.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r6_half_ab
mkdir -p $out
V="auto;block=256,unroll=8,wg_per_cu=1,window=4;block=256,unroll=8,wg_per_cu=2,window=4"
for n in 536870912 1e9 2e9; do
  timeout -k 10 400 python -u tools/op_ab.py --n $n --pairs float16:min,float16:max,bfloat16:min,bfloat16:max \
    --variants "$V" --rounds 4 > $out/n$n.txt 2>&1 || exit $?
  echo "== n=$n"; grep "^|" $out/n$n.txt | tail -n +3
done
