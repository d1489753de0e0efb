export MIREDUCE_FORCE_DEVICE=0
tools/gpu_steps.sh \
 "rehearse2|300|python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29701 bench.py --gpus 2 --backend gloo --steps 20 --warmup 3" \
 "rehearse4|300|python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 4 --backend gloo --steps 20 --warmup 3" \
 "trace_bench|300|rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/trace_r1d -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --trace" \
 "pytest_gpu|900|python -m pytest tests -x -q -m gpu"
