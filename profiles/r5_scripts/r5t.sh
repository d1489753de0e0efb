#!/bin/bash
# Round 5, late: the whole GPU suite, smoke() and the default bench on the committed tree.
set -o pipefail
O=gpurun_out/r5t
mkdir -p $O
st() { echo "$1 rc=$2" | tee -a $O/status.txt; }
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; st pytest_gpu $rc; tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; st smoke $rc; tail -2 $O/smoke.txt; [ $rc -eq 0 ] || exit $rc
s=$(date +%s.%N)
timeout -k 10 600 python3 bench.py --extras-file $O/bench_extras_n1.json > $O/bench.json 2> $O/bench.err
rc=$?; e=$(date +%s.%N); st bench $rc; echo "wall_s=$(python3 -c "print(round($e-$s,1))")" >> $O/status.txt; cat $O/bench.json
exit $rc
