#!/usr/bin/env bash
# Warm vs cold for candidate plans in the 192-384 MB band (32M doubles = 256 MB).
set -euo pipefail
BIN="$(dirname "$0")/../build/bin/reduction"
TMPJ="$(mktemp)"
echo "n,plan,mode,median_ms,GB/s"
for n in 25165824 33554432 46137344; do
for plan in "--threads=512 --unroll=16 --wg-per-cu=1 --policy=default" "--threads=512 --unroll=16 --wg-per-cu=1 --policy=nt" \
            "--threads=256 --unroll=2 --wg-per-cu=3 --policy=nt" "--threads=256 --unroll=4 --wg-per-cu=3 --policy=nt" \
            "--threads=256 --unroll=4 --wg-per-cu=3 --policy=default" "--threads=512 --unroll=8 --wg-per-cu=2 --policy=nt" \
            "--threads=256 --unroll=8 --wg-per-cu=2 --policy=default"; do
  for mode in warm cold; do
    flag=""; [ "$mode" = cold ] && flag="--cold"
    : > "$TMPJ"
    # shellcheck disable=SC2086
    timeout -k 10 120 "$BIN" --method=SUM --type=double --n=$n --iterations=30 --fill=device --noverify \
        --log=none --master-log=none --json="$TMPJ" $flag $plan > /dev/null
    python3 -c "import json,sys; d=json.loads(open('$TMPJ').read().splitlines()[-1]); print(f\"$n,$plan,$mode,{d['median_ms']:.5f},{$n*8/d['median_ms']/1e6:.1f}\")"
  done
done
done
rm -f "$TMPJ"
