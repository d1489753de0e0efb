#!/bin/bash
# Where the single-rank scalar reduce_xgmi run spends its ~5 s (tests/test_apps_gpu.py).
O=gpurun_out/xs; mkdir -p $O
cd "$GRAFT_REPO_ROOT"
for extra in "" "--graph"; do
  s=$(date +%s%N)
  MIREDUCE_LOG_TIMES=1 timeout -k 10 60 ./build/bin/reduce_xgmi --mode=scalar --n=6000007 --dtypes=INT,LONG,FLOAT,DOUBLE \
    --retries=1 --iters=3 $extra > $O/out$extra.txt 2> $O/err$extra.txt || exit $?
  e=$(date +%s%N); echo "scalar $extra: $(( (e - s) / 1000000 )) ms" | tee -a $O/status.txt
done
s=$(date +%s%N)
timeout -k 10 60 ./build/bin/reduce_xgmi --mode=scalar --n=6000007 --dtypes=DOUBLE --ops=SUM --retries=1 --iters=1 > $O/out_min.txt 2> $O/err_min.txt || exit $?
e=$(date +%s%N); echo "scalar one combo: $(( (e - s) / 1000000 )) ms" | tee -a $O/status.txt
s=$(date +%s%N)
timeout -k 10 60 ./build/bin/reduction --method=SUM --type=double --n=6000007 --iterations=1 > $O/out_red.txt 2>&1 || exit $?
e=$(date +%s%N); echo "reduction app one combo: $(( (e - s) / 1000000 )) ms" | tee -a $O/status.txt
