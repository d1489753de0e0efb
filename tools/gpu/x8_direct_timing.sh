#!/bin/bash
O=gpurun_out/x8; mkdir -p $O
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  t0=$(date +%s.%N)
  MIREDUCE_BOOTSTRAP_PORT=29611 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 --master-port 29600 \
    --no-python ./build/bin/reduce_xgmi --mode=vector --collective=direct --ints=4000037 --doubles=2000003 --dtypes=INT,DOUBLE \
    --retries=1 --iters=3 --direct-grid=16 --timeout=30 --graph > $O/out$i.txt 2> $O/err$i.txt
  rc=$?; t1=$(date +%s.%N); echo "run $i rc=$rc wall=$(echo "$t1 - $t0" | bc)" | tee -a $O/status.txt
  [ $rc = 0 ] || exit $rc
done
