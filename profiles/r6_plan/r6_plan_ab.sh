#!/bin/bash
# Round 6: the plan of the widening / 16-bit-compare types. Round 3 moved int32 SUM (int64
# accumulation) and 16-bit MIN / MAX to 256x8x2 with a window of 2 because the window-4, one-workgroup-
# per-CU plan starved on their VALU work (6.1-6.2 TB/s); round 6's fold A/B (profiles/r6_fold/) saw
# the window-4 plan AHEAD for int32 SUM. tools/op_ab.py, 5 interleaved rounds per size, 1 / 4 / 8 GB
# of int32 (and the same element counts of bf16 / fp16).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r6_plan_ab
mkdir -p $out
V="auto;block=256,unroll=8,wg_per_cu=1,window=4"
for n in 268435456 1e9 2e9; do
  timeout -k 10 300 python -u tools/op_ab.py --n $n --pairs int32:sum,bfloat16:max,float16:min --variants "$V" \
    --rounds 5 > $out/n$n.txt 2>&1 || exit $?
  echo "== n=$n"; grep "^|" $out/n$n.txt | tail -n +3
done
