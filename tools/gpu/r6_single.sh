#!/bin/bash
# Round 6: the single-GPU numbers the report figures draw (docs/figures/, tools/report.py): the
# reduction app (the reference's CLI, reduction.cpp) for INT / DOUBLE x MAX / MIN / SUM at 2^28
# elements (BASELINE config 2's size; one JSON each), then a kernel-trace profile of the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r6_single
mkdir -p $out
for t in int double; do
  for m in MAX MIN SUM; do
    timeout -k 10 120 ./build/bin/reduction --method=$m --type=$t --n=268435456 --iterations=100 --log=none \
      --master-log=none --json=$out/${t}_${m}.json > $out/${t}_${m}.txt 2>&1 || exit $?
    tail -3 $out/${t}_${m}.txt
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_prof -o run -- python3 bench.py --steps 20 --warmup 5 \
  > gpurun_out/r6_prof_bench.json 2> gpurun_out/r6_prof_bench.err
