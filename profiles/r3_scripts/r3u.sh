#!/bin/bash
# Round 3, GPU pass U: the fused self-check no longer runs a torch pass over the array right before
# the timed steps. bf16 / f64 bench A/B and the fused-finish GPU tests; then the per-dispatch trace.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3u
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/status.txt
  case $rc in 0|1) ;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
for r in 1 2; do
  step bench_bf16_$r 300 python bench.py --config gpu_4g_bf16_sum --steps 50 --warmup 10 --no-vector-extras --no-candidates
  step bench_f64_$r 300 python bench.py --steps 50 --warmup 10 --no-vector-extras --no-candidates
done
step pytest_xrank 600 python -u -m pytest tests/test_xrank_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread
bash profiles/r3_scripts/r3t.sh
