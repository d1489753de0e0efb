#!/bin/bash
# Round 3, GPU pass AB: the device-side MAXLOC / MINLOC combine (loc_pack, one all-gather,
# loc_pick): its GPU tests, then the MAXLOC config through bench.py twice.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_arg_reduce.py tests/test_apps_gpu.py -m gpu -q -x -k "loc or arg" \
    --timeout 120 --timeout-method thread > $O/pytest.out 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -2 $O/pytest.out
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  timeout -k 10 300 python bench.py --config xgmi_1b_double_maxloc --steps 50 --warmup 10 --no-vector-extras > $O/maxloc_$r.json 2> $O/maxloc_$r.err
  echo "maxloc_$r rc=$?" >> $O/status.txt
done
timeout -k 10 300 python bench.py --config xgmi_1b_double_maxloc --steps 300 --warmup 10 --no-vector-extras --elements 125000000 > $O/maxloc_shard.json 2> $O/maxloc_shard.err
echo "maxloc_shard rc=$?" >> $O/status.txt
