#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp MIREDUCE_FORCE_DEVICE=0 PYTHONFAULTHANDLER=1
mkdir -p gpurun_out/dbg
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --backend gloo --steps 6 --warmup 2 --elements 20000003 --launch graph --collective rccl > gpurun_out/dbg/out.txt 2> gpurun_out/dbg/err.txt
echo rc=$?
grep -v "^\s*frame #" gpurun_out/dbg/err.txt | grep -v "^\s*File \"/usr" | head -90
