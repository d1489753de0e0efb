set -o pipefail
mkdir -p gpurun_out/r1g
O=gpurun_out/r1g
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_apps_gpu.py -q -m gpu -k "bound or step_graph or launch_modes" > $O/pytest_new.txt 2>&1 || { tail -30 $O/pytest_new.txt; exit 1; }
tail -3 $O/pytest_new.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err && cat $O/bench_default.json
for L in graph eager; do timeout -k 10 300 python bench.py --elements 125000000 --steps 400 --warmup 20 --launch $L > $O/bench_125m_$L.json 2> $O/bench_125m_$L.err || exit 1; cat $O/bench_125m_$L.json; done
timeout -k 10 300 python tools/host_overhead.py --steps 400 > $O/host_overhead.jsonl 2> $O/host_overhead.err && cat $O/host_overhead.jsonl
