#!/bin/bash
# Round 5 final-tree check: build() is a no-op here (prebuilt), smoke(), the full GPU suite, and the
# bare `python bench.py` (driver defaults) with its wall time.
set -o pipefail
O=gpurun_out/r5l
mkdir -p $O
st() { echo "$1 rc=$2" | tee -a $O/status.txt; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; st smoke $rc; tail -2 $O/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; st pytest $rc; tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
t0=$(date +%s.%N)
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; t1=$(date +%s.%N); st bench_default $rc
python3 -c "print('wall_s', round($t1 - $t0, 1))" | tee $O/bench_default.wall
cat $O/bench_default.json
exit $rc
