#!/bin/bash
# Round 3, GPU pass G: production-kernel load-window A/B (tools/window_ab.hip) at 8 GB and 1 GB.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3g
mkdir -p $O
for n in 1e9 1.25e8; do
  timeout -k 10 300 ./build/bin/window_ab --n=$n --rounds=7 --iters=20 > $O/window_ab_$n.txt 2>&1
  rc=$?; echo "window_ab_$n rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
