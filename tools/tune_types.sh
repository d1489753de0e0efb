#!/bin/bash
# Re-tune the full reduction at 8 GB for the non-f64 element types (blocks x unrolls x WGs/CU).
set -e
for spec in "float32 2e9" "int32 2e9" "bfloat16 4e9" "int64 1e9"; do
  set -- $spec
  timeout -k 10 200 python tools/tune.py --dtype $1 --op sum --n $2 --blocks 256,512 --unrolls 2,4,8,16 --wgs 1,2,3 \
    --policies nt --rounds 5 --iters 20 --top 8
done
