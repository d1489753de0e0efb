# Kernel durations vs inter-kernel gaps for the N=8 shard size (1 GB/GPU), graph vs eager.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1h
mkdir -p $O
for L in graph eager; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$L -o run --output-format csv -- python3 bench.py --elements 125000000 --steps 200 --warmup 10 --launch $L > $O/bench_$L.json 2> $O/bench_$L.err || exit 1
  python3 tools/kernel_gaps.py $O/trace_$L --bytes 1e9 --skip 20 > $O/gaps_$L.txt && cat $O/gaps_$L.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_hostov -o run --output-format csv -- python3 tools/host_overhead.py --sizes 125000000 --steps 200 --variants eager+ar > $O/hostov.jsonl 2> $O/hostov.err || exit 1
python3 tools/kernel_gaps.py $O/trace_hostov --bytes 1e9 --skip 20 > $O/gaps_eager_ar.txt && cat $O/gaps_eager_ar.txt
