#!/bin/bash
# Repeated headline runs, stderr kept per run (looking for a rare no-output run).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/repro
for i in 1 2 3 4 5 6; do
  t0=$(date +%s.%N)
  timeout -k 10 100 python bench.py --no-vector-extras --collective rccl --steps 100 --no-serial-measure > gpurun_out/repro/out$i.json 2> gpurun_out/repro/err$i.txt
  rc=$?
  t1=$(date +%s.%N)
  echo "run $i rc=$rc wall=$(python -c "print(round($t1-$t0,1))") $(head -c 120 gpurun_out/repro/out$i.json)"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
done
exit 0
