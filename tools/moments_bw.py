#!/usr/bin/env python3
"""Read bandwidth of the fused statistics pass (csrc/kernels/moments.hip) next to the plain
SUM reduction of the same array, per dtype, interleaved rounds in one process.

    python tools/moments_bw.py [--bytes 8e9] [--rounds 5] [--iters 10]

Prints one JSON line per dtype: moments and sum median TB/s (GB = 1e12 B here).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cuda_mpi_reductions_amd._native import native  # noqa: E402
from cuda_mpi_reductions_amd.ops import Reducer, dtype_code, fill_  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--bytes", type=float, default=8e9)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--iters", type=int, default=10)
    a = p.parse_args()
    C = native()
    dev = torch.device("cuda", 0)
    props = torch.cuda.get_device_properties(dev)
    max_grid = 4096
    parts = torch.empty(C.moments_partials_bytes(max_grid), dtype=torch.uint8, device=dev)
    out5 = torch.empty(5, dtype=torch.float64, device=dev)
    red = Reducer(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for dt in (torch.float64, torch.float32, torch.bfloat16, torch.float16):
        n = int(a.bytes) // torch.empty((), dtype=dt).element_size()
        x = torch.empty(n, dtype=dt, device=dev)
        fill_(x, "uniform", seed=3)
        stream = torch.cuda.current_stream(dev).cuda_stream
        acc = torch.empty(1, dtype=torch.float64 if dt == torch.float64 else torch.float32, device=dev)
        if dt == torch.float32:
            acc = torch.empty(1, dtype=torch.float64, device=dev)

        def mom():
            C.moments(x.data_ptr(), n, dtype_code(dt), out5.data_ptr(), parts.data_ptr(), max_grid,
                      props.multi_processor_count, stream)

        def red_sum():
            red(x, "sum", acc.dtype, out=acc)

        times = {"moments": [], "sum": []}
        for _ in range(a.rounds):
            for name, fn in (("moments", mom), ("sum", red_sum)):
                fn()
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) / a.iters)
        k, s, q, mn, mx = out5.tolist()
        ref_mean = x.double().mean().item()
        rec = {"dtype": str(dt).replace("torch.", ""), "n": n, "bytes": n * x.element_size()}
        for name, ts in times.items():
            med = statistics.median(ts)
            rec[f"{name}_ms"] = round(med, 4)
            rec[f"{name}_TBps"] = round(n * x.element_size() / (med * 1e-3) / 1e12, 3)
        rec["mean_ok"] = abs((k + s / n) - ref_mean) <= 1e-9 * max(1.0, abs(ref_mean))
        print(json.dumps(rec), flush=True)
        del x
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
