#!/bin/bash
# Round 3, GPU pass ZA: the peer-map preflight (xrank / direct GPU tests, ranks sharing the GPU),
# reduce_dim GPU tests with the two-batch short-row loop, then the short-row A/B
# (MIREDUCE_DIM_SHORT_PIPE=1 new default vs 0 old loop) over tools/reduce_dim_bw.py's shapes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${PASS:-r3za}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_reduce_dim.py tests/test_xrank_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
for dt in bfloat16 float32; do
  for pipe in 1 0; do
    MIREDUCE_DIM_SHORT_PIPE=$pipe timeout -k 10 300 python -u tools/reduce_dim_bw.py --dtype $dt --rounds 3 > $O/dim_${dt}_pipe$pipe.jsonl 2> $O/dim_${dt}_pipe$pipe.err
    rc=$?; echo "dim $dt pipe$pipe rc=$rc" >> $O/status.txt
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
timeout -k 10 600 python -u -m pytest tests/test_arg_reduce.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_arg.log 2>&1
rc=$?; echo "pytest arg rc=$rc" >> $O/status.txt; tail -2 $O/pytest_arg.log
case $rc in 0) ;; *) exit $rc;; esac
for pipe in 1 0 1 0; do
  MIREDUCE_ARG_SHORT_PIPE=$pipe timeout -k 10 300 python -u tools/arg_reduce_bw.py --only short >> $O/arg_short_pipe$pipe.jsonl 2>> $O/arg_short_pipe$pipe.err
  rc=$?; echo "arg short pipe$pipe rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
