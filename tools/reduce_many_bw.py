#!/usr/bin/env python3
"""Per-tensor L2 norms of a parameter-like list of tensors: ReduceMany (one launch, fused square)
vs torch._foreach_norm and vs a per-tensor torch.linalg.vector_norm loop. The list mimics one
transformer-block-per-entry parameter shard: large matrices plus many small vectors.

    python tools/reduce_many_bw.py [--layers 32] [--hidden 4096] [--dtype bfloat16] [--iters 20]

One JSON line per variant: median ms per call and GB/s of tensor bytes read (GB = 1e9 B).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cuda_mpi_reductions_amd.ops import ReduceMany, fill_  # noqa: E402

DT = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float64": torch.float64}


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--layers", type=int, default=32)
    p.add_argument("--hidden", type=int, default=4096)
    p.add_argument("--dtype", default="bfloat16", choices=sorted(DT))
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--rounds", type=int, default=5)
    a = p.parse_args()
    dt = DT[a.dtype]
    h = a.hidden
    shapes = []
    for _ in range(a.layers):  # attention q,k,v,o + MLP gate, up, down + two norms + biases
        shapes += [(h, h)] * 4 + [(h * 11 // 4, h)] * 2 + [(h, h * 11 // 4)] + [(h,)] * 2 + [(h,)] * 4
    dev = torch.device("cuda", 0)
    ts = []
    for i, s in enumerate(shapes):
        t = torch.empty(s, dtype=dt, device=dev)
        fill_(t.view(-1), "uniform", seed=i)
        ts.append(t)
    nbytes = sum(t.numel() * t.element_size() for t in ts)
    rm = ReduceMany(ts, "sumsq")
    variants = {
        "mireduce_reduce_many": lambda: rm().sqrt(),
        "torch_foreach_norm": lambda: torch._foreach_norm(ts),
        "torch_loop_vector_norm": lambda: [torch.linalg.vector_norm(t) for t in ts],
    }
    ours = rm().sqrt().double()
    ref = torch.stack([torch.linalg.vector_norm(t.double()) for t in ts])
    ok = bool(torch.allclose(ours, ref, rtol=1e-5))
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
    for k, ts_ in times.items():
        med = statistics.median(ts_)
        print(json.dumps({"variant": k, "tensors": len(ts), "bytes": nbytes, "dtype": a.dtype, "ms": round(med, 4),
                          "GBps": round(nbytes / (med * 1e-3) / 1e9, 1), "segments": rm.segments,
                          "matches_fp64_reference": ok}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
