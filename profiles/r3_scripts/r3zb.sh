#!/bin/bash
# Round 3, GPU pass ZB: the end-of-round tree (full GPU suite, smoke(), default bench), then the
# short-row result stores A/B (MIREDUCE_DIM_NT_OUT=1 non-temporal vs 0 plain, pipelined loop).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${PASS:-r3zb}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
for dt in bfloat16 float32; do
  for nt in 1 0 1 0; do
    MIREDUCE_DIM_NT_OUT=$nt timeout -k 10 300 python -u tools/reduce_dim_bw.py --dtype $dt --rounds 3 >> $O/dim_${dt}_nt$nt.jsonl 2>> $O/dim_${dt}_nt$nt.err
    rc=$?; echo "dim $dt nt$nt rc=$rc" >> $O/status.txt
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
