#!/bin/bash
# the new default skew: kernel / fan-in / xrank GPU tests, the N=8 shard bench and the default bench
set -o pipefail
O=gpurun_out/r5am
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fanin_gpu.py tests/test_xrank_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -5 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for k in 1 2; do
  timeout -k 10 300 python3 bench.py --elements 125000000 --steps 50 --warmup 10 --no-vector-extras --extras-file $O/s$k.json > $O/shard$k.json 2> $O/shard$k.err || exit $?
  python3 -c "import json; d=json.load(open('$O/shard$k.json')); print('shard', d['value'], d['ms_per_step'], d['verified'], d['summary']['plans'])"
done
timeout -k 10 600 python3 bench.py --extras-file $O/x.json > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench.json')); print('default', d['value'], d['verified'], d['summary']['plans'])"
