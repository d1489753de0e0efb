#!/bin/bash
# Round 3, GPU pass T: why is the bf16 bench step ~70 us slower than the same kernel in tune.py?
# Kernel trace of the bf16 config's bench run (kernel names, durations, gaps).
O=gpurun_out/r3t
mkdir -p $GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bf16 -o run -- python3 bench.py \
    --config gpu_4g_bf16_sum --steps 20 --warmup 5 --no-vector-extras --no-candidates --launch ${LAUNCH:-auto} > $O/bf16.json 2> $O/bf16.err
echo "bf16 rc=$?" >> $O/status.txt
python3 tools/kernel_gaps.py $O/bf16 --match "reduce_stream" --bytes 8e9 > $O/bf16_gaps.txt 2>&1
find $O/bf16 -name "*kernel_stats.csv" -exec cp {} $O/bf16_kernel_stats.csv \;
python3 - <<'PY' > gpurun_out/r3t/bf16_trace_tail.txt 2>&1
import csv, glob
rows = []
for p in glob.glob("gpurun_out/r3t/bf16/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
prev = None
for r in rows:
    if "reduce_stream" not in r["Kernel_Name"] and "fill_kernel" not in r["Kernel_Name"]:
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = "" if prev is None else f"gap {(s - prev) / 1e3:10.1f} us"
    prev = e
    print(f"{(s - t0) / 1e3:12.1f} us  {(e - s) / 1e3:9.2f} us  {gap}  {r['Kernel_Name'][:110]}")
PY
rm -rf $O/bf16
