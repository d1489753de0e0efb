#!/bin/bash
# Round 5: the r5c experiments, then the GPU suite and the driver's bench command (r5b).
set -o pipefail
bash profiles/r5_scripts/r5c.sh > gpurun_out/r5c_stdout.txt 2>&1
echo "r5c rc=$?"
tail -30 gpurun_out/r5c_stdout.txt
bash profiles/r5_scripts/r5b.sh
