#!/usr/bin/env python3
"""Per-XCD end times of the PRODUCTION streaming kernel (ReduceConfig::debug_wg_stamps).

tools/wg_timeline.hip times re-implementations of the body; this asks the shipped kernel itself:
every workgroup stamps the wall clock after its last streamed tile was consumed, plus its XCC id
and tile count. For each size, ``--launches`` back-to-back launches run on one stream and the last
one's stamps are read; repeated ``--rounds`` times. Printed per round: the spread of workgroup end
times (min / p50 / p99 / max, us relative to the earliest end) and the mean end per XCC — a
systematic per-XCD pattern would be the case for an XCD-weighted static split; a random one is
not. The stamped launch is not timed (the kernel-only time per launch is, from hipEvents).

    python tools/xcd_balance.py --sizes 125000000,1000000000 --rounds 5
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
    ap.add_argument("--sizes", default="125000000,1000000000", help="element counts")
    ap.add_argument("--dtype", default="float64", choices=("float64", "float32", "bfloat16", "int64", "int32"))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--json", default=None, help="append one JSON object per (size, round)")
    ap.add_argument("--skews", default=None,
                    help="comma list of XCD skews (permille, MIREDUCE_XCD_SKEW) measured interleaved in every "
                         "round on the same array (default: the plan's own)")
    ap.add_argument("--offset-tiles", type=int, default=0,
                    help="start the array this many 32 KB tiles into its allocation (address-residue test)")
    ap.add_argument("--stream", choices=("current", "new"), default="current",
                    help="launch on torch's current stream or on a new one (another hardware queue)")
    a = ap.parse_args(argv)
    C = native()
    dev = torch.device("cuda", 0)
    red = Reducer(dev)
    dt = getattr(torch, a.dtype)
    acc = default_acc_dtype(dt, "sum")
    out = torch.zeros(1, dtype=acc, device=dev)
    stream = torch.cuda.current_stream(dev) if a.stream == "current" else torch.cuda.Stream(dev)
    skews = [None] if a.skews is None else [int(v) for v in a.skews.split(",")]
    off = a.offset_tiles * (32768 // torch.empty(0, dtype=dt).element_size())  # 32 KB tiles
    for n in (int(float(x)) for x in a.sizes.split(",")):
        base = torch.empty(n + off, dtype=dt, device=dev)
        x = base[off:]
        fill_(x, "uniform" if dt.is_floating_point else "fullrange", seed=11)
        stamps = torch.zeros(3 * red.ws.max_grid, dtype=torch.int64, device=dev)

        def launch(st=0):
            return C.reduce(red.ws, x.data_ptr(), n, dtype_code(x.dtype), op_code("sum"), dtype_code(acc),
                            out.data_ptr(), stream.cuda_stream, wg_stamps=st)
        for r, sk in ((r, sk) for r in range(a.rounds) for sk in skews):
            if sk is None:
                os.environ.pop("MIREDUCE_XCD_SKEW", None)
            else:
                os.environ["MIREDUCE_XCD_SKEW"] = str(sk)
            plan = launch()
            grid = plan["grid"]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.launches):
                launch()
            e1.record(stream)
            launch(stamps.data_ptr())
            torch.cuda.synchronize()
            us_per = e0.elapsed_time(e1) * 1e3 / a.launches
            st = stamps[: 3 * grid].view(grid, 3).cpu()
            end = (st[:, 0] - st[:, 0].min()).double() / TICKS_PER_US
            xcc = st[:, 1]
            srt = end.sort().values
            # XCC of workgroup b minus b % 8: one constant when the dispatcher deals round-robin
            rot = ((xcc - torch.arange(grid)) % 8).tolist()
            per = {int(k): round(float(end[xcc == k].mean()), 2) for k in sorted(set(xcc.tolist()))}
            row = {"n": n, "dtype": a.dtype, "round": r, "skew": sk, "xskew": plan.get("xskew"), "offset_tiles": a.offset_tiles, "stream": a.stream,
                   "xcc_rotation": {int(k): rot.count(k) for k in sorted(set(rot))},
                   "base_mod_2mb": int(x.data_ptr() % (2 << 20)), "grid": grid, "us_per_launch": round(us_per, 2),
                   "end_spread_us": {"p50": round(float(srt[grid // 2]), 2),
                                     "p99": round(float(srt[int(0.99 * (grid - 1))]), 2),
                                     "max": round(float(srt[-1]), 2)},
                   "mean_end_by_xcc_us": per, "tiles": sorted(set(st[:, 2].tolist())),
                   "plan": {k: plan[k] for k in ("block", "unroll", "window", "nontemporal")}}
            print(json.dumps(row), flush=True)
            if a.json:
                with open(a.json, "a") as f:
                    f.write(json.dumps(row) + "\n")
        del x, base
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
