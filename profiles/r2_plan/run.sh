#!/bin/bash
# Is 512x8x1 consistently ahead of the default 512x16x1 for large f64 on this round's boxes?
# Interleaved head-to-head at 8 GB and 4 GB (f64 SUM) and 8 GB int64 MAX, nt loads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_plan
mkdir -p $O
timeout -k 10 400 python -u tools/tune.py --dtype float64 --op sum --ns 500000000,1000000000 --rounds 12 --iters 20 \
  --blocks 256,512 --unrolls 8,16 --wgs 1 --policies nt > $O/h2h_f64.txt 2>&1 || { tail -20 $O/h2h_f64.txt; exit 1; }
grep -v "^\[tune\]" $O/h2h_f64.txt
timeout -k 10 300 python -u tools/tune.py --dtype int64 --op max --ns 1000000000 --rounds 8 --iters 20 \
  --blocks 512 --unrolls 8,16 --wgs 1 --policies nt > $O/h2h_i64.txt 2>&1 || { tail -20 $O/h2h_i64.txt; exit 1; }
grep -v "^\[tune\]" $O/h2h_i64.txt
