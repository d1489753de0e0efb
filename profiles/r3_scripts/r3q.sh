#!/bin/bash
# Round 3, GPU pass Q: the op-aware 4-/2-byte defaults (profiles/r3_types/). (1) kernel GPU tests
# incl. the new default-plan tests; (2) reduction-app A/B of the new default against the old one
# (f32 SUM / int32 SUM / f32 MAX at 8 GB, bf16 SUM via bench), 3 interleaved rounds; (3) every
# BASELINE.json GPU config through bench.py, incl. the HBM-filling fp32 SUM.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3q
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  case $rc in 0|1) ;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
step pytest 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_half.py tests/test_plan.py -m gpu -q -x \
    --timeout 120 --timeout-method thread
B=./build/bin/reduction
C="--fill=device --iterations=20 --log=none --master-log=none"
for r in 1 2 3; do
  step f32sum_new_$r 120 $B --method=SUM --type=float --n=2000000000 $C --json=$O/ab.jsonl
  step f32sum_old_$r 120 $B --method=SUM --type=float --n=2000000000 $C --threads=512 --unroll=4 --wg-per-cu=1 --window=0 --json=$O/ab.jsonl
  step i32sum_new_$r 120 $B --method=SUM --type=int --n=2000000000 $C --json=$O/ab.jsonl
  step i32sum_old_$r 120 $B --method=SUM --type=int --n=2000000000 $C --threads=512 --unroll=4 --wg-per-cu=1 --window=0 --json=$O/ab.jsonl
  step f32max_new_$r 120 $B --method=MAX --type=float --n=2000000000 $C --json=$O/ab.jsonl
  step f32max_old_$r 120 $B --method=MAX --type=float --n=2000000000 $C --threads=512 --unroll=4 --wg-per-cu=1 --window=0 --json=$O/ab.jsonl
done
O=$O/configs bash profiles/r2_configs/run.sh > $O/configs_summary.txt 2>&1
echo "configs rc=$?" >> $O/status.txt
exit 0
