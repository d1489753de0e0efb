#!/bin/bash
# Round 5: does a HIP runtime setting move the 1.6 us per-launch floor? tools/launch_floor.hip under
# each setting, 2 interleaved rounds (graph-replayed back-to-back launches, median of 5 x 200).
set -o pipefail
O=gpurun_out/r5i
mkdir -p $O
SETTINGS=("" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=0" "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0" "DEBUG_HIP_KERNARG_COPY_OPT=0")
for r in 1 2; do
  for i in "${!SETTINGS[@]}"; do
    s="${SETTINGS[$i]}"
    tag="s${i}_r$r"
    echo "== $tag: ${s:-default}" > $O/$tag.txt
    if [ -n "$s" ]; then
      timeout -k 10 120 env $s ./build/bin/launch_floor --rounds=5 --launches=200 >> $O/$tag.txt 2>&1
    else
      timeout -k 10 120 ./build/bin/launch_floor --rounds=5 --launches=200 >> $O/$tag.txt 2>&1
    fi
    rc=$?; echo "$tag rc=$rc" >> $O/status.txt
    [ $rc -le 1 ] || exit $rc
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, os, re, sys, collections
rows = collections.defaultdict(dict)
for f in sorted(glob.glob(sys.argv[1] + "/s*_r*.txt")):
    lines = open(f).read().splitlines()
    name = lines[0].split(": ", 1)[1]
    for ln in lines:
        m = re.match(r"(\S+)\s+([\d.]+)\s+([\d.]+)", ln)
        if m and not ln.startswith("variant"):
            rows[name].setdefault(m.group(1), []).append(float(m.group(2)))
vars_ = ["empty1", "poll768", "reduce_1024", "reduce_16777216", "reduce_125000000"]
print("%-36s" % "setting" + "".join("%18s" % v for v in vars_))
for name, d in rows.items():
    print("%-36s" % name + "".join("%18s" % "/".join("%.2f" % x for x in d.get(v, [])) for v in vars_))
PY
cat $O/summary.txt
