#!/bin/bash
# Round 3, GPU pass C: r1-vs-r3 regression A/B, HBM-fill sizes + PMC, (XCD, residue) affinity sweep.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/regress.sh || exit $?
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/hbmfill.sh || exit $?
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_shift
mkdir -p $O
for n in 1.25e8 1e9; do
  timeout -k 10 300 ./build/bin/wg_timeline --set=shift --n=$n --rounds=3 --iters=10 > $O/shift_$n.txt 2>&1
  rc=$?; echo "shift_$n rc=$rc" >> $O/status.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
du -sh gpurun_out
