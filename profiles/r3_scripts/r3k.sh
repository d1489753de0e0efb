#!/bin/bash
# Round 3, GPU pass K: explicit-window sweeps for the other element types (bf16 8 GB, int32 8 GB)
# on the production kernels, then every BASELINE.json GPU config through bench.py.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_input_preserved_gpu.py -x -v --timeout 120 --timeout-method thread \
    > $O/pytest_preserved.log 2>&1
rc=$?; echo "pytest_preserved rc=$rc" >> $O/status.txt; tail -2 $O/pytest_preserved.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/tune.py --dtype bfloat16 --n 4000000000 --blocks 256,512 --unrolls 2,4,8 --wgs 1,2 \
    --policies nt --windows 0,2,4 --rounds 3 --iters 10 --json $O/tune_bf16.json > $O/tune_bf16.txt 2>&1
rc=$?; echo "tune_bf16 rc=$rc" >> $O/status.txt
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/tune.py --dtype int32 --n 2000000000 --blocks 256,512 --unrolls 2,4,8 --wgs 1,2 \
    --policies nt --windows 0,2,4 --rounds 3 --iters 10 --json $O/tune_i32.json > $O/tune_i32.txt 2>&1
rc=$?; echo "tune_i32 rc=$rc" >> $O/status.txt
case $rc in 0) ;; *) exit $rc;; esac
O=gpurun_out/r3k/configs bash profiles/r2_configs/run.sh > $O/configs_summary.txt 2>&1
rc=$?; echo "configs rc=$rc" >> $O/status.txt
exit $rc
