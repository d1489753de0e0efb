set -e
for w in 1 2 3 4 6 8; do
  echo "=== WG $w"
  MIREDUCE_DIM_WG_PER_CU=$w timeout -k 10 120 python tools/reduce_dim_bw.py --dtype bfloat16 --rounds 3 --iters 5
done
