#!/bin/bash
# Round 3, GPU pass S: bf16 SUM 8 GB, new plan vs old, in bench.py (graph-replayed fused steps) and
# in tools/tune.py (eager back-to-back launches) on ONE box: pass R's bench gave 7133 GB/s where
# pass P's tune gave 7376 on another box.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  case $rc in 0|1) ;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
for r in 1 2; do
  step bench_new_$r 300 python bench.py --config gpu_4g_bf16_sum --steps 50 --warmup 10 --no-vector-extras --no-candidates
  step bench_old_$r 300 python bench.py --config gpu_4g_bf16_sum --steps 50 --warmup 10 --no-vector-extras --no-candidates \
      --block 256 --unroll 4 --wg-per-cu 2
  step bench_f64_$r 300 python bench.py --steps 50 --warmup 10 --no-vector-extras --no-candidates --no-plan-tune
done
step tune_bf16 300 python -u tools/tune.py --dtype bfloat16 --n 4e9 --blocks 256 --unrolls 4,8 --wgs 1,2 --policies nt \
    --windows 0,4 --rounds 5 --iters 10
