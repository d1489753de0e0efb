#!/bin/bash
# Round 4: run-to-run variance of the default bench on one box (3 back-to-back runs of the driver's
# N=1 command), then the same through torch.distributed.run with one rank (the driver's launcher).
O=${O:-gpurun_out/r4_var}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err
  rc=$?; echo "bench_$i rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 > $O/bench_torchrun.json 2> $O/bench_torchrun.err
echo "bench_torchrun rc=$?" >> $O/status.txt
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(os.path.basename(f), d["value"], d["ms_per_step"], d["launcher"], d["config"]["kernel_plan"]["xskew"],
          d["plan_tuning"]["chosen"], d["verified"])
PY
cat $O/summary.txt
