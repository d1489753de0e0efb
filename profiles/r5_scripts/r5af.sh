#!/bin/bash
# after the rebuild: smoke, the kernel / fan-in / xrank GPU tests, the default bench
set -o pipefail
O=gpurun_out/r5af
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
tail -1 $O/smoke.txt
timeout -k 10 900 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fanin_gpu.py tests/test_xrank_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -5 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 600 python3 bench.py --extras-file $O/x.json > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['verified'], d['native_source_hash'])"
