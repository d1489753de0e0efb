# A/B of the single-pass fan-in shape (tree = two-level, flat = final arriver folds all).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1r
mkdir -p $O
MIREDUCE_FANIN=flat timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x > $O/pytest_flat.txt 2>&1 || { tail -30 $O/pytest_flat.txt; exit 1; }
tail -1 $O/pytest_flat.txt
for rep in 1 2 3; do
  for F in tree flat; do
    MIREDUCE_FANIN=$F timeout -k 10 120 python bench.py --elements 125000000 --steps 400 --warmup 20 > $O/b1g_${F}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/b1g_${F}_$rep.json')); print('1GB', '$F', d['value'], d['ms_per_step'], d['verified'], d['config']['kernel_plan']['flat'])"
  done
done
for F in tree flat; do
  MIREDUCE_FANIN=$F timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr_$F -o run --output-format csv -- build/bin/reduction --method=SUM --type=double --n=125000000 --iterations=100 --fill=device --noverify --log=none --master-log=none > /dev/null 2>&1 || exit 1
  echo "== $F"; python3 tools/kernel_gaps.py $O/tr_$F --bytes 1e9 --skip 5
  MIREDUCE_FANIN=$F timeout -k 10 200 rocprofv3 --kernel-trace -d $O/trs_$F -o run --output-format csv -- build/bin/reduction --method=SUM --type=double --n=1048576 --iterations=100 --fill=device --noverify --log=none --master-log=none > /dev/null 2>&1 || exit 1
  echo "== $F small 8MB"; python3 tools/kernel_gaps.py $O/trs_$F --bytes 8388608 --skip 5
done
for rep in 1 2; do
  for F in tree flat; do
    MIREDUCE_FANIN=$F timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/b8g_${F}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/b8g_${F}_$rep.json')); print('8GB', '$F', d['value'], d['ms_per_step'], d['verified'])"
  done
done
