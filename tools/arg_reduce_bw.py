#!/usr/bin/env python3
"""Arg-reduction bandwidth: arg_reduce (csrc/kernels/arg_reduce.hip) vs torch.argmax / torch.max(dim)
on whole arrays, vocabulary-style long rows and router-style short rows.

    python tools/arg_reduce_bw.py [--iters 20] [--rounds 5] [--only whole|rows|short]
    python tools/arg_reduce_bw.py --sweep   # long-row kernel: unroll x resident workgroups per CU

One JSON line per (shape, dtype, variant): median ms and GB/s of input bytes read (GB = 1e9 B).
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
from cuda_mpi_reductions_amd.ops import arg_reduce, fill_  # noqa: E402
from cuda_mpi_reductions_amd.ops.reduce import DTYPE_CODES  # noqa: E402

CASES = [  # (kind, rows, cols, dtype)
    ("whole", 1, 1_000_000_000, torch.float64),
    ("whole", 1, 1_000_000_000, torch.float32),
    ("whole", 1, 2_000_000_000, torch.bfloat16),
    ("whole", 1, 500_000_000, torch.int32),
    ("rows", 1024, 131_072, torch.bfloat16),   # logits of 1024 tokens over a 128k vocabulary
    ("rows", 64, 262_144, torch.float32),
    ("rows", 8, 16_777_216, torch.bfloat16),
    ("rows", 65_536, 4096, torch.float32),     # medium rows: a wave per row
    ("rows", 262_144, 2048, torch.bfloat16),
    ("rows", 8192, 8192, torch.float32),
    ("short", 4_194_304, 64, torch.bfloat16),  # router logits: 4M tokens over 64 experts
    ("short", 2_097_152, 256, torch.bfloat16),
    ("short", 1_048_576, 128, torch.float32),
    ("short", 16_777_216, 8, torch.float32),
]


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--only", choices=["whole", "rows", "short"])
    p.add_argument("--sweep", action="store_true")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    if a.sweep:
        return sweep(a, dev)
    for kind, rows, cols, dt in CASES:
        if a.only and kind != a.only:
            continue
        x = torch.empty(rows * cols, dtype=dt, device=dev)
        if dt.is_floating_point:
            fill_(x, "uniform", seed=rows + cols)
        else:
            fill_(x, "fullrange", seed=rows + cols)
        x = x.view(rows, cols) if kind != "whole" else x
        dim = None if kind == "whole" else 1
        nbytes = x.numel() * x.element_size()
        if kind == "whole":
            variants = {"mireduce_arg_reduce": lambda: arg_reduce(x, "max"),
                        "torch_argmax": lambda: torch.argmax(x),
                        "torch_max_value_only": lambda: torch.max(x)}
        else:
            variants = {"mireduce_arg_reduce": lambda: arg_reduce(x, "max", dim),
                        "torch_max_dim": lambda: torch.max(x, dim)}
        ours = arg_reduce(x, "max", dim)[1]
        ref = torch.argmax(x) if dim is None else torch.argmax(x, dim)
        ok = bool(torch.equal(ours, ref))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        times = {k: [] for k in variants}
        for _ in range(a.rounds):
            for k, fn in variants.items():
                fn()
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / a.iters)
        for k, ts in times.items():
            med = statistics.median(ts)
            print(json.dumps({"kind": kind, "rows": rows, "cols": cols, "dtype": str(dt).replace("torch.", ""),
                              "variant": k, "ms": round(med, 4), "GBps": round(nbytes / (med * 1e-3) / 1e9, 1),
                              "matches_torch_argmax": ok}), flush=True)
        del x
        torch.cuda.empty_cache()
    return 0


def sweep(a, dev) -> int:
    C = native()
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    stream = torch.cuda.current_stream(dev).cuda_stream
    for kind, rows, cols, dt in CASES:
        if kind == "short":
            continue
        x = torch.empty(rows * cols, dtype=dt, device=dev)
        fill_(x, "uniform" if dt.is_floating_point else "fullrange", seed=rows + cols)
        v = torch.empty(rows, dtype=dt, device=dev)
        i = torch.empty(rows, dtype=torch.int64, device=dev)
        scratch = torch.zeros(max(C.arg_reduce_scratch_bytes(rows, cols, DTYPE_CODES[dt], ncu), 1), dtype=torch.uint8,
                              device=dev)
        ref = torch.argmax(x.view(rows, cols), 1)
        nbytes = x.numel() * x.element_size()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for unroll in (2, 4, 8):
            for wg in (1, 2, 3, 4, 6, 8):
                def run():
                    return C.arg_reduce_rows(x.data_ptr(), rows, cols, DTYPE_CODES[dt], 2, v.data_ptr(), i.data_ptr(),
                                             scratch.data_ptr(), ncu, stream, unroll, wg)
                plan = run()
                ok = bool(torch.equal(i, ref))
                ts = []
                for _ in range(a.rounds):
                    e0.record()
                    for _ in range(a.iters):
                        run()
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) / a.iters)
                med = statistics.median(ts)
                print(json.dumps({"kind": kind, "rows": rows, "cols": cols, "dtype": str(dt).replace("torch.", ""),
                                  "unroll": unroll, "wg_per_cu": plan["wg_per_cu"], "grid": plan["grid"],
                                  "splits": plan["splits"], "ms": round(med, 4),
                                  "GBps": round(nbytes / (med * 1e-3) / 1e9, 1), "ok": ok}), flush=True)
        del x
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
