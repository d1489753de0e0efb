#!/bin/bash
# Round 4: int32 SUM in production with dot2 half-sums on the window-4 plan + XCD skew 20. The new
# GPU tests first (exactness incl. the periodic fold), then the full GPU suite, smoke and the
# default bench, then the reduction app: the new default vs the old plan shape (256x8x2 window 2,
# now also with dot2 half-sums), 3 interleaved rounds, 8 GB.
O=gpurun_out/r4_i32b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "int32_sum_dot2 or more_than_2_pow_31 or all_combos" > $O/pytest_new.txt 2>&1
rc=$?; echo "pytest_new rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
one() {  # one <tag> <skew or -> <args...>
  local tag=$1 sk=$2; shift 2
  if [ "$sk" = "-" ]; then unset MIREDUCE_XCD_SKEW; else export MIREDUCE_XCD_SKEW=$sk; fi
  timeout -k 10 120 ./build/bin/reduction --method=SUM --type=int --n=2e9 --fill=device --iterations=60 \
      --timing=batch --log=none --master-log=none --json=$O/$tag.jsonl "$@" > $O/$tag.out 2>&1
  local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || { tail -3 $O/$tag.out; exit $rc; }
}
for r in 1 2 3; do
  one "new_$r" -
  one "w2x2_$r" - --unroll=8 --wg-per-cu=2 --threads=256 --window=2
  one "w4x1s0_$r" 0 --unroll=8 --wg-per-cu=1 --threads=256 --window=4
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*_[123].jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    acc[os.path.basename(f)[:-6].rsplit("_", 1)[0]].append((d["avg_ms"] * 1e3, d["gb_per_s"], d["verified"], d["window"], d["grid"]))
for tag, v in sorted(acc.items()):
    print(f"{tag:8s} us {' '.join('%.2f' % x[0] for x in sorted(v)):26s} best GB/s {max(x[1] for x in v):8.1f} verified {all(x[2] for x in v)} window {v[0][3]} grid {v[0][4]}")
PY
cat $O/summary.txt
