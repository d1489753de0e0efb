#!/usr/bin/env python3
"""Per-dispatch durations and gaps of the last timed window in a rocprofv3 database of bench.py
(profiles/r5_window/): are the first steps of a window slower than the rest, and by how much?
The window is the last run of back-to-back `reduce_stream` dispatches (split at idle gaps > 1 ms)
with at least --k dispatches.
    usage: tools/window_kernels.py <results.db> [--k 20]"""
import argparse
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_db import kernels  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("db")
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--needle", default="reduce_stream")
    a = ap.parse_args(argv)
    ks = [(s, e) for n, s, e in kernels(a.db) if a.needle in n]
    runs, cur = [], []
    for s, e in ks:
        if cur and s - cur[-1][1] > 1_000_000:
            runs.append(cur)
            cur = []
        cur.append((s, e))
    if cur:
        runs.append(cur)
    runs = [r for r in runs if len(r) >= a.k]
    if not runs:
        print("no window found")
        return 1
    last = runs[-1][-a.k:]  # the timed window: the last K dispatches of the last run
    d = [(e - s) / 1e3 for s, e in last]
    g = [(last[i][0] - last[i - 1][1]) / 1e3 for i in range(1, len(last))]
    print(f"timed window (last {a.k}): durations us {', '.join(f'{x:.1f}' for x in d)}")
    print(f"  gaps us {', '.join(f'{x:.2f}' for x in g)}")
    print(f"  span {(last[-1][1] - last[0][0]) / 1e3:.1f} us; first 3 mean {sum(d[:3]) / 3:.1f}, "
          f"rest median {sorted(d[3:])[len(d[3:]) // 2]:.1f}")
    for idx, w in enumerate(runs[-3:]):
        print(f"run {idx}: {len(w)} dispatches")
        durs = [(e - s) / 1e3 for s, e in w]
        gaps = [(w[i][0] - w[i - 1][1]) / 1e3 for i in range(1, len(w))]
        head = ", ".join(f"{d:.1f}" for d in durs[:6])
        tail = sorted(durs[6:])
        med = tail[len(tail) // 2] if tail else float("nan")
        print(f"  first 6 durations us: {head}; median of the rest {med:.1f}")
        print(f"  gaps us: first 5 {', '.join(f'{g:.2f}' for g in gaps[:5])}; median {sorted(gaps)[len(gaps) // 2]:.2f}")
        print(f"  window span {(w[-1][1] - w[0][0]) / 1e3:.1f} us = {(w[-1][1] - w[0][0]) / 1e3 / len(w):.2f} us per step")
    return 0


if __name__ == "__main__":
    sys.exit(main())
