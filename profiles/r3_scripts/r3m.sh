#!/bin/bash
# Round 3, GPU pass M: the node-preset sweep at P=1 (failed in pass L: bench under torchrun rc=1),
# with every point's stdout/stderr kept, then the same bench command directly.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 600 python -u tools/sweep.py --preset node --ranks 1 --out $O/node --timeout 300 -- \
    --ints=1000003 --doubles=1000003 --retries=1 > $O/sweep.log 2>&1
rc=$?; echo "sweep rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 50 --warmup 10 > $O/bench_torchrun.json 2> $O/bench_torchrun.err
rc=$?; echo "bench_torchrun rc=$rc" >> $O/status.txt
exit 0
