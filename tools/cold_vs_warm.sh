#!/usr/bin/env bash
# Warm (Infinity-Cache resident on repeat) vs cold (--cold: 1 GiB scratch overwrite before each
# iteration) bandwidth of the single-pass kernel for n = 2^17 .. 2^30 doubles.
#   usage: tools/cold_vs_warm.sh OUT.csv
set -euo pipefail
OUT="$1"
BIN="$(dirname "$0")/../build/bin/reduction"
echo "n,bytes,mode,avg_ms,GB/s" > "$OUT"
for k in $(seq 17 30); do
  n=$((1 << k))
  for mode in warm cold; do
    flag=""; [ "$mode" = cold ] && flag="--cold"
    line=$(timeout -k 10 120 "$BIN" --method=SUM --type=double --n=$n --iterations=20 --fill=device --noverify \
           --log=none --master-log=none $flag | grep "Reduction, Throughput")
    gbs=$(echo "$line" | sed -E 's/.*Throughput = ([0-9.]+) GB\/s, Time = ([0-9.]+) s.*/\1/')
    t=$(echo "$line" | sed -E 's/.*Time = ([0-9.]+) s.*/\1/')
    echo "$n,$((n * 8)),$mode,$(python3 -c "print($t*1e3)"),$gbs" >> "$OUT"
  done
done
cat "$OUT"
