#!/bin/bash
# Round 3, GPU pass ZC: the N=8 per-GPU shard (125M doubles = 1 GB) through bench.py, 300 serial
# steps, plain and under rocprofv3 --kernel-trace --stats (end-of-session tree).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3zc
mkdir -p $O
timeout -k 10 300 python -u bench.py --elements 125000000 --steps 300 --warmup 20 --no-vector-extras > $O/shard.json 2> $O/shard.err
rc=$?; echo "shard rc=$rc" >> $O/status.txt
case $rc in 0) ;; *) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --elements 125000000 --steps 300 --warmup 20 --no-vector-extras > $O/shard_prof.json 2> $O/shard_prof.err
echo "prof rc=$?" >> $O/status.txt
