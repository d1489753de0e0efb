B=build/bin
tools/gpu_steps.sh \
 "pytest_gpu|900|python -m pytest tests/test_kernels_gpu.py -x -q" \
 "red_cfg2|300|cd gpurun_out && ../$B/reduction --method=SUM --type=double --n=268435456 --qatest --json=reduction.jsonl --log=reduction_cfg2.txt" \
 "red_cfg3|300|cd gpurun_out && ../$B/reduction --method=MIN --type=int64 --n=268435456 --pattern=fullrange --qatest --json=reduction.jsonl --log=reduction_cfg3.txt" \
 "red_ref_default|300|cd gpurun_out && ../$B/reduction --method=SUM --qatest --json=reduction.jsonl --log=none && ../$B/reduction --method=MAX --type=float --cpufinal --qatest --log=none && ../$B/reduction --method=MIN --type=double --kernel=6 --maxblocks=64 --qatest --log=none --json=reduction.jsonl" \
 "bandwidth|300|$B/bandwidth_test --host --json=gpurun_out/bandwidth.jsonl" \
 "xgmi_scalar1|300|$B/reduce_xgmi --mode=scalar --n=1000000000 --dtypes=DOUBLE --ops=SUM --retries=3 --iters=20 --json=gpurun_out/xgmi.jsonl && $B/reduce_xgmi --mode=scalar --n=1000000000 --dtypes=DOUBLE --ops=SUM --retries=3 --iters=20 --graph" \
 "xgmi_vector1|300|$B/reduce_xgmi --mode=vector --ints=16M --doubles=8M --retries=2 --json=gpurun_out/xgmi.jsonl" \
 "tune_f64|600|python tools/tune.py --dtype float64 --op sum --n 1e9 --rounds 5 --iters 10 --json gpurun_out/tune_f64_sum.json" \
 "tune_i64min|600|python tools/tune.py --dtype int64 --op min --n 268435456 --rounds 5 --iters 10 --blocks 256,512 --unrolls 2,4,8 --wgs 0,4,8 --json gpurun_out/tune_i64_min.json" \
 "shmoo|600|cd gpurun_out && ../$B/reduction --method=SUM --type=double --shmoo --iterations=20 --log=none > shmoo_double_sum.csv"
