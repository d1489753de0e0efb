#!/bin/bash
# Default bench (serial measured with the fused finish when it passed), wall time of the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_serial_fused
mkdir -p $O
s=$SECONDS
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
echo "bench wall $((SECONDS - s)) s"
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(d['value'], d['config']['collective'], d.get('serial_gbps'), d.get('serial_collective'), d.get('collective_tuning'))"
