#!/bin/bash
# per-XCC end times of the production kernel at the 1 GB shard and 8 GB with the round-5 default skew
set -o pipefail
mkdir -p gpurun_out/r5ap
timeout -k 10 300 python3 -u tools/xcd_balance.py --sizes 125000000,1000000000 --rounds 3 --launches 20 \
  --json gpurun_out/r5ap/xcd.jsonl > gpurun_out/r5ap/xcd.txt 2>&1
rc=$?; tail -12 gpurun_out/r5ap/xcd.txt; exit $rc
