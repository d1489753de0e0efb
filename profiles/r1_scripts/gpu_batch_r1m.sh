# Full GPU suite + cold/warm sweep with the new plan + default bench.
set -o pipefail
O=gpurun_out/r1m
mkdir -p $O
timeout -k 10 1500 python -m pytest tests -q -m gpu -x > $O/pytest_gpu_full.txt 2>&1 || { tail -40 $O/pytest_gpu_full.txt; exit 1; }
tail -3 $O/pytest_gpu_full.txt
timeout -k 10 400 bash tools/cold_vs_warm.sh $O/cold_vs_warm.csv > /dev/null && cat $O/cold_vs_warm.csv
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && cat $O/bench_default.json
