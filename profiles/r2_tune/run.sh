#!/bin/bash
# Kernel-parameter sweep at the N=4 and N=2 shards of the headline (2 GB, 4 GB per GPU) and the
# N=1 size (8 GB), float64 SUM, nt loads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2_tune
mkdir -p $O
timeout -k 10 600 python -u tools/tune.py --dtype float64 --op sum --ns 250000000,500000000,1000000000 --rounds 5 --iters 20 \
  --blocks 256,512 --unrolls 2,4,8,16 --wgs 1,2,3 --policies nt --json $O/tune.json > $O/tune.txt 2>&1 || { tail -20 $O/tune.txt; exit 1; }
grep -v "^\[tune\]" $O/tune.txt
