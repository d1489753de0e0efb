#!/usr/bin/env bash
# Warm (Infinity-Cache resident on repeat) vs cold (--cold: 1 GiB scratch overwrite before each
# iteration) bandwidth of the single-pass kernel for n = 2^17 .. 2^30 doubles.
#   usage: tools/cold_vs_warm.sh OUT.csv [extra reduction flags...]
set -euo pipefail
OUT="$1"; shift
BIN="$(dirname "$0")/../build/bin/reduction"
TMPJ="$(mktemp)"
echo "n,bytes,mode,avg_ms,median_ms,GB/s,block,unroll,grid" > "$OUT"
for k in $(seq 17 30); do
  n=$((1 << k))
  for mode in warm cold; do
    flag=""; [ "$mode" = cold ] && flag="--cold"
    : > "$TMPJ"
    timeout -k 10 120 "$BIN" --method=SUM --type=double --n=$n --iterations=20 --fill=device --noverify \
        --log=none --master-log=none --json="$TMPJ" $flag "$@" > /dev/null
    python3 - "$TMPJ" "$n" "$mode" >> "$OUT" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
n = int(sys.argv[2]); p = d
print(f"{n},{n*8},{sys.argv[3]},{d['avg_ms']:.5f},{d['median_ms']:.5f},{n*8/d['median_ms']/1e6:.1f},"
      f"{p.get('block','')},{p.get('unroll','')},{p.get('grid','')}")
PY
  done
done
rm -f "$TMPJ"
cat "$OUT"
