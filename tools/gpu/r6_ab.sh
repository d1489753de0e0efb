#!/bin/bash
# Round 6: same-box interleaved A/B against the round-5 tree (abtmp/r5: bench.py + its package with the
# statically linked round-5 extension, built from commit 0b34402 by `make python`), same plan on both
# sides (--no-plan-tune: the tuned default), headline steps only, 3 rounds alternating:
#   * VERDICT r5 item 2 — the pruned production kernel, 1e9-double SUM (the headline);
#   * VERDICT r5 item 5 — BASELINE config 3, 256M int64 MIN (round 6 folds the two elements of a
#     16-byte vector into two accumulators for 8-byte integer MIN / MAX), and int64 SUM as its yardstick;
# then tools/op_ab.py on the new tree: int64 MIN / SUM, fp64 SUM under the tuned plan and two
# waves-per-SIMD / window candidates for MIN.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r6_ab
mkdir -p $out
common="--steps 100 --warmup 10 --no-vector-extras --no-candidates --no-decompose --no-plan-tune"
run() {  # side config round
  if [ $1 = old ]; then b=abtmp/r5/bench.py; else b=bench.py; fi
  MIREDUCE_EXTRAS_DIR=$out timeout -k 10 240 python -u $b $common --config $2 > $out/$2_$1_$3.json 2> $out/$2_$1_$3.err || exit $?
  echo "$2 $1 $3 $(python -c "import json; d=[json.loads(l) for l in open('$out/$2_$1_$3.json') if l.startswith('{')][0]; print(d['value'], d['ms_per_step'], d['verified'])")"
}
for cfg in xgmi_1b_double_sum gpu_256m_int64_min; do
  for r in 1 2 3; do
    if [ $((r % 2)) = 1 ]; then run old $cfg $r; run new $cfg $r; else run new $cfg $r; run old $cfg $r; fi
  done
done
timeout -k 10 300 python -u tools/op_ab.py --n 268435456 --pairs int64:min,int64:sum,float64:sum \
  --variants "auto;wg_per_cu=2;block=512,unroll=8,window=4" --rounds 5 > $out/op_ab.txt 2>&1
