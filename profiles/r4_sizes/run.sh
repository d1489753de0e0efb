#!/bin/bash
# Round 4 final kernel: f64 SUM bandwidth vs array size (128 MB .. 128 GB), kernel-only batch timing
# (back-to-back launches) and the reference's per-iteration timing, 2 interleaved rounds, verified.
set -o pipefail
O=${O:-gpurun_out/r4_sizes}
mkdir -p $O
one() {  # one <tag> <args...>
  local tag=$1; shift
  timeout -k 10 300 ./build/bin/reduction --method=SUM --type=double --fill=device --log=none --master-log=none \
      --json=$O/$tag.jsonl "$@" > $O/$tag.out 2>&1
  local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -3 $O/$tag.out; exit $rc; }
}
for r in 1 2; do
  for n in 16777216 134217728 1000000000 4000000000 16000000000; do
    it=60; [ $n -ge 4000000000 ] && it=10
    one "batch_${n}_$r" --n=$n --iterations=$it --timing=batch
    one "periter_${n}_$r" --n=$n --iterations=$it --timing=per-iter
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    mode, n, _ = os.path.basename(f)[:-6].split("_")
    acc[(mode, int(n))].append((d["median_ms"] * 1e3, d["gb_per_s"], d["verified"], d["grid"], d["window"]))
for (mode, n), v in sorted(acc.items(), key=lambda kv: (kv[0][0], kv[0][1])):
    print(f"{mode:8s} n={n:12d} ({n * 8 / 1e9:7.2f} GB) median us {' '.join('%.2f' % x[0] for x in v):24s} "
          f"GB/s {' '.join('%.1f' % x[1] for x in v):18s} verified {all(x[2] for x in v)} grid {v[0][3]} window {v[0][4]}")
PY
cat $O/summary.txt
