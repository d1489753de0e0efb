#!/bin/bash
# The 1-3 GB band for 8-byte types (N=8 / N=4 shards): the current 256x2x3 against 256x4x2,
# 256x8x1, 256x2x4 and 512x2x2 / 512x4x1 (f64 SUM, 1 GB and 2 GB, 10 interleaved rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_plan6
mkdir -p $O
timeout -k 10 600 python -u tools/tune.py --dtype float64 --op sum --ns 125000000,250000000 --rounds 10 --iters 40 \
  --blocks 256,512 --unrolls 2,4,8 --wgs 1,2,3,4 --policies nt --top 10 > $O/band.txt 2>&1 || { tail -20 $O/band.txt; exit 1; }
grep -v "^\[tune\]" $O/band.txt
