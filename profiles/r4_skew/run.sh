#!/bin/bash
# Round 4: XCD skew per element type / op with the anchored split (reduction app, one process per
# point, kernel-only batch timing, 8 GB per reduction, 2 interleaved rounds). Which plans want a
# skew besides the 8-/4-byte window-4 SUM plans it is on for? (The two-pass launches now anchor the
# split too, so the app's two-launch oracle for bf16 sums matches a skewed run's order again.)
set -o pipefail
O=${O:-gpurun_out/r4_skew}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_fanin_gpu.py > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
one() {  # one <tag> <skew> <args...>
  local tag=$1; export MIREDUCE_XCD_SKEW=$2; shift 2
  timeout -k 10 120 ./build/bin/reduction "$@" --fill=device --iterations=60 --timing=batch --log=none \
      --master-log=none --json=$O/$tag.jsonl > $O/$tag.out 2>&1
  local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -3 $O/$tag.out; exit $rc; }
}
for r in 1 2; do
  for sk in 0 10 20 30; do
    one "i32sum_s${sk}_$r" $sk --method=SUM --type=int --n=2e9
    one "i32max_s${sk}_$r" $sk --method=MAX --type=int --n=2e9
    one "bf16sum_s${sk}_$r" $sk --method=SUM --type=bf16 --n=4e9
    one "f64max_s${sk}_$r" $sk --method=MAX --type=double --n=1e9
    one "i64min_s${sk}_$r" $sk --method=MIN --type=int64 --n=1e9
    one "f32sum_s${sk}_$r" $sk --method=SUM --type=float --n=2e9
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[os.path.basename(f)[:-6].rsplit("_", 1)[0]].append((d["avg_ms"] * 1e3, d["gb_per_s"], d["verified"], d["window"], d["grid"]))
for tag, v in sorted(acc.items()):
    print(f"{tag:14s} us {' '.join('%.2f' % x[0] for x in sorted(v)):28s} best GB/s {max(x[1] for x in v):8.1f} "
          f"verified {all(x[2] for x in v)} window {v[0][3]} grid {v[0][4]}")
PY
cat $O/summary.txt
