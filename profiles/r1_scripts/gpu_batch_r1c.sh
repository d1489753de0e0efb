B=build/bin
tools/gpu_steps.sh \
 "pytest_gpu|900|python -m pytest tests -x -q -m gpu" \
 "smoke|300|python -c \"import __graft_entry__ as g; g.smoke()\"" \
 "bench_default|300|python bench.py" \
 "bench_serial|300|python bench.py --serial" \
 "bench_1gb_shard|300|python bench.py --elements 125000000 --steps 200 --warmup 20" \
 "xgmi_scalar_graph|300|$B/reduce_xgmi --mode=scalar --n=1000000000 --dtypes=DOUBLE --ops=SUM,MIN,MAX --retries=3 --iters=20 --graph --json=gpurun_out/xgmi_r1c.jsonl" \
 "red_cfg2|300|cd gpurun_out && ../$B/reduction --method=SUM --type=double --n=268435456 --qatest --json=reduction_r1c.jsonl --log=none" \
 "red_cfg3|300|cd gpurun_out && ../$B/reduction --method=MIN --type=int64 --n=268435456 --pattern=fullrange --qatest --json=reduction_r1c.jsonl --log=none" \
 "prof_trace|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1c -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5" \
 "prof_pmc|300|rocprofv3 --pmc FETCH_SIZE SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_r1c -o run --output-format csv -- $B/reduction --method=SUM --type=double --n=1000000000 --fill=device --iterations=10 --noverify --log=none"
