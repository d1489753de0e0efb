#!/bin/bash
# Polled fan-in (default) vs ticketed flat fan-in: numerics first, then kernel-only times per size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r2_small2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py tests/test_xrank_gpu.py -k "not eight and not share and not extras and not corrupt and not missing and not fallback" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for mode in poll flat; do
  for n in 1024 65536 1048576 4194304 16777216 125000000 1000000000; do
    MIREDUCE_FANIN=$mode timeout -k 10 120 rocprofv3 --kernel-trace -d $O/${mode}_$n -o t -- ./build/bin/reduction --method=SUM --type=double --n=$n --iterations=60 --timing=batch --log=none --fill=device > $O/${mode}_$n.log 2>&1 || exit 1
  done
done
echo done
