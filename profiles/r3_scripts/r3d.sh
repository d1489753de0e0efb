#!/bin/bash
# Round 3, GPU pass D: kernel-only fan-in / tree A/B against the round-1 tree, the per-wave dynamic
# tail experiment (wg_timeline --set=wavetail) at 8 GB and 1 GB, HBM-fill sizes + PMC at 292 GB.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/fanin_ab.sh || exit $?
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_wavetail
mkdir -p $O
for n in 1e9 1.25e8; do
  timeout -k 10 300 ./build/bin/wg_timeline --set=wavetail --n=$n --rounds=5 --iters=10 > $O/wavetail_$n.txt 2>&1
  rc=$?; echo "wavetail_$n rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/hbmfill.sh
du -sh gpurun_out
