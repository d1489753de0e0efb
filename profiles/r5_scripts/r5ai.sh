#!/bin/bash
# run-to-run spread of the default bench on one box: 6 back-to-back processes (driver's K=20 W=5 and the default K=50 W=10)
set -o pipefail
O=gpurun_out/r5ai
mkdir -p $O
for i in 1 2 3; do
  for kw in "20 5" "50 10"; do
    set -- $kw
    timeout -k 10 300 python3 bench.py --steps $1 --warmup $2 --no-vector-extras --extras-file $O/x.json > $O/b_${i}_$1.json 2> $O/b_${i}_$1.err || exit $?
    python3 -c "import json; d=json.load(open('$O/b_${i}_$1.json')); print('run $i K=$1', d['value'], d['ms_per_step'], d['verified'], d['summary']['plans'])"
  done
done | tee $O/summary.txt
