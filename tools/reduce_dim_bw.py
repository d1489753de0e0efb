#!/usr/bin/env python3
"""Read bandwidth of reduce_dim (csrc/kernels/reduce_dim.hip) vs PyTorch's own reduction of the
same tensor along the same axis (x.sum(dim, dtype=acc) / amax), interleaved rounds in one process.

    python tools/reduce_dim_bw.py [--gb 4] [--rounds 5] [--iters 10] [--dtype float32]

One JSON line per (shape, dim, op): mireduce and torch median ms and TB/s (GB = 1e12 B here).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cuda_mpi_reductions_amd.ops import default_acc_dtype, fill_, reduce_dim  # noqa: E402

DT = {"float32": torch.float32, "float64": torch.float64, "bfloat16": torch.bfloat16, "int32": torch.int32}


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--gb", type=float, default=4.0)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--dtype", default="float32", choices=sorted(DT))
    a = p.parse_args()
    dt = DT[a.dtype]
    es = torch.empty((), dtype=dt).element_size()
    n = int(a.gb * 1e9) // es
    dev = torch.device("cuda", 0)
    flat = torch.empty(n, dtype=dt, device=dev)
    fill_(flat, "uniform" if dt.is_floating_point else "smallint", seed=11)
    cases = []
    for cols in (8, 64, 4096, 1 << 16, 1 << 22):
        rows = n // cols
        for dim in (1, 0):
            for op in ("sum", "max"):
                cases.append(((rows, cols), dim, op))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for shape, dim, op in cases:
        x = flat[: shape[0] * shape[1]].view(shape)
        acc = default_acc_dtype(dt, op)

        def ours():
            return reduce_dim(x, op, dim)

        def theirs():
            return x.sum(dim, dtype=acc) if op == "sum" else x.amax(dim)

        times = {"mireduce": [], "torch": []}
        ok = True
        for _ in range(a.rounds):
            for name, fn in (("mireduce", ours), ("torch", theirs)):
                r = fn()
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) / a.iters)
                if name == "mireduce":
                    ref = theirs().to(r.dtype)
                    if op == "sum" and r.dtype.is_floating_point:
                        ok = ok and bool(torch.allclose(r.double(), ref.double(), rtol=1e-5, atol=1e-6))
                    else:
                        ok = ok and bool(torch.equal(r, ref))
        nbytes = shape[0] * shape[1] * es
        rec = {"dtype": a.dtype, "shape": list(shape), "dim": dim, "op": op, "bytes": nbytes, "match": ok}
        for name, ts in times.items():
            med = statistics.median(ts)
            rec[f"{name}_ms"] = round(med, 4)
            rec[f"{name}_TBps"] = round(nbytes / (med * 1e-3) / 1e12, 3)
        rec["speedup"] = round(rec["torch_ms"] / rec["mireduce_ms"], 3)
        print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
