#!/bin/bash
# Round 5, final tree after the skew default: the whole GPU suite, smoke(), the default bench and every BASELINE config.
set -o pipefail
O=gpurun_out/r5an
mkdir -p $O
st() { echo "$1 rc=$2" | tee -a $O/status.txt; }
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; st pytest_gpu $rc; tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; st smoke $rc; tail -1 $O/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --extras-file $O/bench_extras_n1.json > $O/bench.json 2> $O/bench.err
rc=$?; st bench $rc; cat $O/bench.json; [ $rc -eq 0 ] || exit $rc
O=$O/configs timeout -k 10 1200 bash tools/gpu/configs.sh > $O/configs_summary.txt 2>&1
rc=$?; st configs $rc; cat $O/configs_summary.txt
exit $rc
