#!/bin/bash
# Round 5: A/B of the kernel-body refactor (reduce_stream -> reduce_stream_body + wrappers) and of the
# PIN prologue: launch_floor built from the previous commit (launch_floor_ref) vs this tree, 3
# alternating runs each; this tree's binary also times the *_pin variants.
set -o pipefail
O=gpurun_out/r5j
mkdir -p $O
for r in 1 2 3; do
  for b in launch_floor_ref launch_floor; do
    timeout -k 10 180 ./build/bin/$b --rounds=5 --launches=200 > $O/${b}_$r.txt 2>&1
    rc=$?; echo "${b}_$r rc=$rc" >> $O/status.txt
    [ $rc -le 1 ] || exit $rc
  done
done
python3 - "$O" <<'PY' > $O/summary.txt
import glob, os, re, sys, collections
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/launch_floor*_*.txt")):
    b = os.path.basename(f).rsplit("_", 1)[0]
    for ln in open(f):
        m = re.match(r"(\S+)\s+([\d.]+)\s+([\d.]+)", ln)
        if m and not ln.startswith("variant"):
            rows[m.group(1)][b].append(float(m.group(2)))
print("%-28s %-30s %-30s" % ("variant", "ref (previous commit)", "this tree"))
for v, d in rows.items():
    print("%-28s %-30s %-30s" % (v, " ".join("%.3f" % x for x in d.get("launch_floor_ref", [])),
                                  " ".join("%.3f" % x for x in d.get("launch_floor", []))))
PY
cat $O/summary.txt
