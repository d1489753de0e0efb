#!/usr/bin/env python3
"""Why does the HBM-filling reduction (BASELINE config 5: fp32 SUM over ~292 GB on one GPU) stream
~3-4 % slower than the same kernel over 8 GB? (profiles/r3_hbmfill/ found
+35 % DRAM-credit stalls per request, not translation.)

One hypothesis is positional drift: the interleaved split gives workgroup b the tiles b, b + grid,
..., so all workgroups start in one narrow window, but a workgroup that streams 1-2 % faster runs
ahead — over 292 GB by GBs — and the concurrently read addresses spread over many DRAM rows. An
8 GB launch cannot drift that far. This tool measures, on ONE array filling most of HBM, in
interleaved rounds:

* ``whole``: one launch over the whole array (``segment_bytes=-1``: the round-4 plan);
* ``seg<G>``: the library's segmented launches (ReduceConfig::segment_bytes = G GiB): the same
  bytes as back-to-back launches over G-GiB segments, the earlier results carried into the last
  launch — same total work, bounded drift (``seg8`` is the round-5 default above 16 GiB);
* ``slice<k>``: one 8 GB launch at the array's start / middle / end (is some region of HBM slower?);

plus the per-workgroup end-time spread of the whole-array launch (ReduceConfig::debug_wg_stamps:
how far the workgroups drifted apart by the end). All results are checked against the whole-array
value. GB = 1e9 B.

    python tools/hbm_chunks.py --fraction 0.9 --rounds 3 --segments 4,8,16
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cuda_mpi_reductions_amd._native import native  # noqa: E402
from cuda_mpi_reductions_amd.ops import Reducer, default_acc_dtype, dtype_code, fill_, op_code  # noqa: E402

TICKS_PER_US = 100.0  # gfx950 wall clock: 100 MHz


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--fraction", type=float, default=0.9, help="of the free HBM to fill")
    ap.add_argument("--elements", type=float, default=0, help="array size in elements (overrides --fraction)")
    ap.add_argument("--slices", action=argparse.BooleanOptionalAction, default=True,
                    help="also time 8 GB slices at the start / middle / end")
    ap.add_argument("--stamps", action=argparse.BooleanOptionalAction, default=True,
                    help="also read the whole-array launch's per-workgroup end stamps")
    ap.add_argument("--dtype", default="float32", choices=("float32", "float64"))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--segments", default="4,8,16", help="segment sizes in GiB (comma list; fractions allowed)")
    ap.add_argument("--reps", type=int, default=1, help="back-to-back reductions per timed sample")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    C = native()
    dev = torch.device("cuda", 0)
    dt = getattr(torch, a.dtype)
    es = torch.empty(0, dtype=dt).element_size()
    free, _ = torch.cuda.mem_get_info(dev)
    n = int(a.elements) if a.elements else int(free * a.fraction) // es
    if not a.elements:
        n -= n % 4096
    x = torch.empty(n, dtype=dt, device=dev)
    fill_(x, "uniform", seed=5)
    acc = default_acc_dtype(dt, "sum")
    red = Reducer(dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    gb = n * es / 1e9
    print(f"[hbm] {n} {a.dtype} = {gb:.1f} GB", flush=True)
    segs = [float(v) for v in a.segments.split(",") if v]
    outs = torch.zeros(4096, dtype=acc, device=dev)

    def launch(view, out, **kw):
        kw.setdefault("segment_bytes", -1)
        return C.reduce(red.ws, view.data_ptr(), view.numel(), dtype_code(dt), op_code("sum"), dtype_code(acc),
                        out.data_ptr(), s, **kw)

    def timed(fn) -> float:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        ev0.record()
        fn()
        ev1.record()
        torch.cuda.synchronize(dev)
        return ev0.elapsed_time(ev1) * 1e-3

    launch(x, outs[:1])  # warm-up
    torch.cuda.synchronize(dev)
    ref = float(outs[0].item())
    tol = 1e-6 * abs(ref) + 1e-3

    results = {}
    slice_n = int(8e9) // es
    slices = {"slice_start": 0, "slice_mid": (n // 2) - (n // 2) % 4096, "slice_end": n - slice_n} \
        if a.slices and n >= 2 * slice_n else {}
    for r in range(a.rounds):
        R = a.reps
        t = timed(lambda: [launch(x, outs[:1]) for _ in range(R)]) / R
        ok = abs(float(outs[0].item()) - ref) <= tol
        results.setdefault("whole", []).append((gb / t, ok))
        for g in segs:
            t = timed(lambda: [launch(x, outs[:1], segment_bytes=int(g * (1 << 30))) for _ in range(R)]) / R
            results.setdefault(f"seg{g:g}", []).append((gb / t, abs(float(outs[0].item()) - ref) <= tol))
        for name, off in slices.items():
            v = x[off:off + slice_n]
            t = timed(lambda: launch(v, outs[:1]))
            results.setdefault(name, []).append((slice_n * es / 1e9 / t, True))
        launch(x, outs[:1])
    spread, by_xcc, plan = {}, {}, None
    if not a.stamps:
        return _report(a, n, gb, plan, results, spread, by_xcc)
    # end-time spread of the whole-array launch's workgroups
    stamps = torch.zeros(3 * red.ws.max_grid, dtype=torch.int64, device=dev)
    plan = launch(x, outs[:1], wg_stamps=stamps.data_ptr())
    torch.cuda.synchronize(dev)
    g = plan["grid"]
    st = stamps[:3 * g].view(g, 3).cpu()
    ends = (st[:, 0] - st[:, 0].min()).double() / TICKS_PER_US
    e = ends.sort().values
    spread = {"grid": g, "min": 0.0, "p50": float(e[g // 2]), "p99": float(e[int(0.99 * (g - 1))]), "max": float(e[-1])}
    by_xcc = {}
    for xcc in sorted(set(st[:, 1].tolist())):
        m = st[:, 1] == xcc
        by_xcc[int(xcc)] = round(float(ends[m].mean()), 1)
    return _report(a, n, gb, plan, results, spread, by_xcc)


def _report(a, n, gb, plan, results, spread, by_xcc) -> int:
    out = {"n": n, "dtype": a.dtype, "gb": round(gb, 2), "plan": plan, "rounds": a.rounds,
           "gbps": {k: [round(v, 1) for v, _ in vs] for k, vs in results.items()},
           "verified": all(ok for vs in results.values() for _, ok in vs),
           "wg_end_spread_us": spread, "wg_end_mean_by_xcc_us": by_xcc}
    for k, vs in results.items():
        print(f"[hbm] {k:12s} GB/s {' '.join('%.1f' % v for v, _ in vs)}  verified {all(ok for _, ok in vs)}")
    if spread:
        print(f"[hbm] whole-array workgroup end spread (us after the first): p50 {spread['p50']:.0f} "
              f"p99 {spread['p99']:.0f} max {spread['max']:.0f}; mean by XCC {by_xcc}")
    if a.json:
        with open(a.json, "a") as f:
            f.write(json.dumps(out) + "\n")
    return 0 if out["verified"] else 1


if __name__ == "__main__":
    sys.exit(main())
