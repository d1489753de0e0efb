#!/bin/bash
# The window's fixed cost with the fused-bound step (bench.py's headline kernel) vs the plain one
set -o pipefail
mkdir -p gpurun_out/r5z
timeout -k 10 300 python3 -u tools/window_overhead.py --elements 125000000 --steps 20,200 --variants bench,plain \
  --rounds 9 --json gpurun_out/r5z/plain.json > gpurun_out/r5z/plain.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/window_overhead.py --elements 125000000 --steps 20,200 --variants bench,plain \
  --rounds 9 --fused --json gpurun_out/r5z/fused.json > gpurun_out/r5z/fused.txt 2>&1
