#!/bin/bash
# Head-to-head of the top points at 4 GB and 8 GB (10 rounds), to pick the >= 3 GB default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2_tune2
mkdir -p $O
timeout -k 10 600 python -u tools/tune.py --dtype float64 --op sum --ns 500000000,1000000000 --rounds 10 --iters 20 \
  --blocks 256,512 --unrolls 8,16 --wgs 1 --policies nt --json $O/tune_f64.json > $O/tune_f64.txt 2>&1 || { tail -20 $O/tune_f64.txt; exit 1; }
grep -v "^\[tune\]" $O/tune_f64.txt
timeout -k 10 600 python -u tools/tune.py --dtype int64 --op max --ns 1000000000 --rounds 6 --iters 20 \
  --blocks 256,512 --unrolls 8,16 --wgs 1 --policies nt > $O/tune_i64.txt 2>&1 || { tail -20 $O/tune_i64.txt; exit 1; }
grep -v "^\[tune\]" $O/tune_i64.txt
