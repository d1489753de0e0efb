#!/bin/bash
# same-box A/B of the round-1 tree (4cc6ac6, built in .ab/r1) against this tree on
# the driver's exact command, interleaved, 3 runs each, under rocprofv3 --kernel-trace --stats.
O=${O:-$GRAFT_REPO_ROOT/gpurun_out/regress}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2 3; do
  for tree in r1 r3; do
    if [ $tree = r1 ]; then cd "$GRAFT_REPO_ROOT/.ab/r1"; else cd "$GRAFT_REPO_ROOT"; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${tree}_$i -o run -- python3 bench.py --gpus 1 --steps 20 \
        --warmup 5 > $O/${tree}_$i.json 2> $O/${tree}_$i.err
    rc=$?
    echo "${tree}_$i rc=$rc" | tee -a $O/status.txt
    # keep gpurun_out small (<= 64 MiB merged back): summaries only, the databases stay on the box
    (cd "$GRAFT_REPO_ROOT" && python3 tools/ab_kernels.py $O/${tree}_$i/run_results.db > $O/${tree}_$i.kernels.md 2>&1; \
     python3 tools/prof_db.py $O/${tree}_$i/run_results.db > $O/${tree}_$i.stats.txt 2>&1; rm -rf $O/${tree}_$i)
    case $rc in 0|1) ;; *) echo "stopping (rc=$rc)"; exit $rc;; esac
  done
done
