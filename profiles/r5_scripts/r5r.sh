#!/bin/bash
# The driver's 8-rank command shape, every extra on, ranks sharing the one GPU (gloo: RCCL cannot put
# two ranks on one device). Wall time against the 420 s run budget; the line and the sidecar.
set -o pipefail
mkdir -p gpurun_out/r5r
export MIREDUCE_FORCE_DEVICE=0
s=$(date +%s.%N)
timeout -k 10 560 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 8 --backend gloo --extras-file gpurun_out/r5r/bench_extras_n8.json \
  > gpurun_out/r5r/line.json 2> gpurun_out/r5r/stderr.txt
rc=$?
e=$(date +%s.%N)
echo "rc=$rc wall_s=$(python -c "print(round($e-$s,1))")" > gpurun_out/r5r/wall.txt
cat gpurun_out/r5r/wall.txt
exit $rc
