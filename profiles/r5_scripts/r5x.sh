#!/bin/bash
# Split the timed window's fixed cost (tools/window_overhead.py) at the N=8 shard
set -o pipefail
mkdir -p gpurun_out/r5x
timeout -k 10 300 python3 -u tools/window_overhead.py --elements 125000000 --steps 20,200 --variants bench,bench_nosync,barrier --rounds 9 \
  --json gpurun_out/r5x/window.json > gpurun_out/r5x/window.txt 2>&1
