# Failure-detection GPU tests, graph tests (thread-local capture), cold/warm sweep.
set -o pipefail
O=gpurun_out/r1j
mkdir -p $O
timeout -k 10 700 python -m pytest tests/test_apps_gpu.py tests/test_kernels_gpu.py -q -m gpu -k "corrupt or lost_peer or cold or step_graph or bound or launch_modes" > $O/pytest_fault.txt 2>&1 || { tail -40 $O/pytest_fault.txt; exit 1; }
tail -3 $O/pytest_fault.txt
timeout -k 10 400 bash tools/cold_vs_warm.sh $O/cold_vs_warm.csv
