#!/bin/bash
# Round 6: within-box spread of the driver's command (5 back-to-back runs on one box), next to the
# box-to-box spread of profiles/r6_final/ (7249-7349 GB/s over five boxes).
O=gpurun_out/r6_spread; mkdir -p $O
cd "$GRAFT_REPO_ROOT"
for i in 1 2 3 4 5; do
  timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-vector-extras > $O/run$i.json 2> $O/run$i.err || exit $?
  python3 -c "import json;d=json.loads(open('$O/run$i.json').read().strip().splitlines()[-1]);s=d['summary'];print($i,d['value'],d['ms_per_step'],d['verified'],s.get('local_gbps'),s.get('plans'))" | tee -a $O/summary.txt
done
