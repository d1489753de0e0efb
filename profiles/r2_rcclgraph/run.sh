#!/bin/bash
# N=1 bench with the RCCL combine under rocprofv3: the replayed graph must show the RCCL
# AllReduce kernel after every reduce_stream dispatch (VERDICT r1 item 1 "done looks like").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_rcclgraph
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 bench.py --collective rccl --steps 20 --warmup 4 --no-vector-extras --no-serial-measure > $O/bench_rccl.json 2> $O/bench_rccl.err || exit $?
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
