#!/bin/bash
# SIGSEGV in the 2-rank gloo capture-fallback bench: Python stack via faulthandler, and the same
# run without the reduce.c extras.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONFAULTHANDLER=1 MIREDUCE_FORCE_DEVICE=0
O=gpurun_out/r2_serial_fused
mkdir -p $O
A="--gpus 2 --backend gloo --steps 6 --warmup 2 --elements 20000003 --launch graph --collective rccl"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29611 bench.py $A --no-vector-extras > $O/noextras.out 2> $O/noextras.err
echo "no extras rc=$?"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29612 bench.py $A > $O/extras.out 2> $O/extras.err
echo "extras rc=$?"
grep -n "File \|Fatal\|Segmentation" $O/extras.err | head -60 || true
