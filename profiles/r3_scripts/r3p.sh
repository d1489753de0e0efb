#!/bin/bash
# Round 3, GPU pass P: the window sweep at the 1 GB band (bf16 / f32 / int32 SUM) and for the
# non-widening ops at 8 GB (int32 MAX, f32 MAX, f16 MAX), before moving the 4- and 2-byte defaults.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3p
mkdir -p $O
for spec in "bfloat16 5e8 sum" "float32 2.5e8 sum" "int32 2.5e8 sum" "int32 2e9 max" "float32 2e9 max" "float16 4e9 max" "bfloat16 1e9 sum"; do
  set -- $spec
  timeout -k 10 400 python -u tools/tune.py --dtype $1 --n $2 --op $3 --blocks 256,512 --unrolls 2,4,8 --wgs 1,2,3 \
      --policies nt --windows 0,2,4 --rounds 5 --iters 10 --json $O/tune_$1_$2_$3.json > $O/tune_$1_$2_$3.txt 2>&1
  rc=$?; echo "tune_$1_$2_$3 rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
