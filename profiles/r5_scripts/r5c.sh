#!/bin/bash
# Round 5: (1) small arrays — is the warm re-read of 2^24 doubles served from the MALL with the
# default (non-nt) policy, and where is the per-launch floor; (2) the HBM-filling config: whole-array
# launch vs chunked launches vs 8 GB slices, and the workgroups' end-time drift; (3) a one-GPU dry
# run of tools/sweep.py --rccl-knobs (reduce_xgmi over RCCL, 12 knob settings, world 1).
set -o pipefail
O=gpurun_out/r5c
mkdir -p $O
echo start > $O/status.txt
O=$O/small N=16777216 ROUNDS=2 PLANS="--threads=256 --unroll=4 --wg-per-cu=3 --window=0 --policy=nt;--threads=256 --unroll=4 --wg-per-cu=3 --window=0 --policy=default" bash tools/gpu/plan_sweep.sh > /dev/null || exit $?
O=$O/small64 N=8388608 ROUNDS=2 PLANS="--threads=256 --unroll=4 --wg-per-cu=3 --window=0 --policy=nt;--threads=256 --unroll=4 --wg-per-cu=3 --window=0 --policy=default" bash tools/gpu/plan_sweep.sh > /dev/null || exit $?
O=$O/small32 N=4194304 ROUNDS=2 PLANS="--threads=256 --unroll=4 --wg-per-cu=3 --window=0 --policy=nt;--threads=256 --unroll=4 --wg-per-cu=3 --window=0 --policy=default" bash tools/gpu/plan_sweep.sh > /dev/null || exit $?
O=$O/floor N=1024 ROUNDS=2 PLANS="--threads=256 --unroll=4 --wg-per-cu=3 --window=0" bash tools/gpu/plan_sweep.sh > /dev/null || exit $?
echo "small done" >> $O/status.txt
timeout -k 10 300 python3 tools/hbm_chunks.py --fraction 0.9 --rounds 3 --chunks 8,32 --json $O/hbm_chunks.jsonl > $O/hbm_chunks.txt 2>&1
rc=$?; echo "hbm_chunks rc=$rc" >> $O/status.txt; cat $O/hbm_chunks.txt | grep "^\[hbm\]"
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 tools/sweep.py --rccl-knobs --ranks 1 --out $O/knobs --timeout 120 -- --ints=16M --doubles=8M --retries=2 > $O/knobs.txt 2>&1
rc=$?; echo "knobs rc=$rc" >> $O/status.txt; tail -20 $O/knobs.txt
exit $rc
