#!/bin/bash
# Interleaved A/B of the fan-in at the headline size (8 GB f64), bench.py --collective rccl, 100 steps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2 3; do
  for mode in poll flat; do
    MIREDUCE_FANIN=$mode timeout -k 10 120 python bench.py --no-vector-extras --collective rccl --steps 100 --no-serial-measure 2>>gpurun_out/ab_err.txt \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', d['value'], d['ms_per_step'])" || exit 1
  done
done
for mode in poll flat; do
  MIREDUCE_FANIN=$mode timeout -k 10 120 python bench.py --no-vector-extras --collective rccl --steps 100 --no-serial-measure --elements 125000000 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode 1GB', d['value'], d['ms_per_step'])" || exit 1
done
