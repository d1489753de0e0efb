#!/bin/bash
# the default bench line after the config / summary additions
set -o pipefail
O=gpurun_out/r5ad
mkdir -p $O
timeout -k 10 600 python3 bench.py --extras-file $O/bench_extras_n1.json > $O/bench.json 2> $O/bench.err
rc=$?; cat $O/bench.json; wc -c $O/bench.json; exit $rc
