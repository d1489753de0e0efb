#!/bin/bash
# Round 3, GPU pass X: the explicit load window in the long-row arg-reduction kernel: its GPU tests,
# an interleaved window A/B on whole arrays, and the MAXLOC config through bench.py.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_arg_reduce.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_arg.out 2>&1
rc=$?; echo "pytest_arg rc=$rc" >> $O/status.txt; tail -2 $O/pytest_arg.out
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/arg_reduce_bw.py --window-ab --rounds 5 --iters 10 > $O/window_ab.jsonl 2> $O/window_ab.err
echo "window_ab rc=$?" >> $O/status.txt
for r in 1 2; do
  timeout -k 10 300 python bench.py --config xgmi_1b_double_maxloc --steps 50 --warmup 10 --no-vector-extras > $O/maxloc_$r.json 2> $O/maxloc_$r.err
  echo "maxloc_$r rc=$?" >> $O/status.txt
done
