#!/bin/bash
# reduce_many A/B: segment size (MIREDUCE_MANY_SEG_KB) x resident workgroups per CU
# (MIREDUCE_MANY_WG_PER_CU), tools/reduce_many_bw.py on the 13 GB transformer-like list.
set -e
DT=${1:-bfloat16}
for kb in 64 256 1024 4096; do
  for w in 1 2 4 8; do
    echo "=== SEG ${kb}KB WG $w $DT"
    MIREDUCE_MANY_SEG_KB=$kb MIREDUCE_MANY_WG_PER_CU=$w timeout -k 10 120 python tools/reduce_many_bw.py --dtype $DT --rounds 3 --iters 10
  done
done
