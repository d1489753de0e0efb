"""Fused one-pass statistics: count, sum, mean, variance, std, min, max of a float tensor
(fp32 / fp64 / bf16 / fp16 storage; all statistics are computed in fp64).

Device tensors: one streaming HIP pass (csrc/kernels/moments.hip) computing Σ(x-K), Σ(x-K)²,
min and max with K = x[0] (shifted-data variance), then a one-workgroup fold. Pattern reference:
the fused Σx/Σx² reduction of the vendored MonteCarlo sample (MonteCarlo_reduction.cuh:20-63).
Across ranks (``moments(x, group=...)``) the per-rank raw moments are combined exactly with the
pairwise (Chan et al.) update after an all-gather of 4 values per rank.
"""
from __future__ import annotations

import math

import torch

from .._native import native
from .reduce import dtype_code

__all__ = ["moments", "combine_moments"]


def _raw(x: torch.Tensor):
    """(n, mean, M2, min, max) of one tensor."""
    n = x.numel()
    if n == 0:
        return 0, 0.0, 0.0, math.inf, -math.inf
    if x.device.type == "cuda":
        C = native()
        if x.data_ptr() % 16:
            x = x.clone()
        props = torch.cuda.get_device_properties(x.device)
        max_grid = 4096
        parts = torch.empty(C.moments_partials_bytes(max_grid), dtype=torch.uint8, device=x.device)
        out = torch.empty(5, dtype=torch.float64, device=x.device)
        C.moments(x.data_ptr(), n, dtype_code(x.dtype), out.data_ptr(), parts.data_ptr(), max_grid,
                  props.multi_processor_count, torch.cuda.current_stream(x.device).cuda_stream)
        k, s, q, mn, mx = out.tolist()
    else:
        xd = x.double()
        k = float(xd[0])
        d = xd - k
        s, q = float(d.sum()), float((d * d).sum())
        mn, mx = float(xd.min()), float(xd.max())
    mean = k + s / n
    m2 = max(q - s * s / n, 0.0)
    return n, mean, m2, mn, mx


def combine_moments(a, b):
    """Chan et al. pairwise combination of (n, mean, M2, min, max) tuples."""
    na, ma, qa, mna, mxa = a
    nb, mb, qb, mnb, mxb = b
    n = na + nb
    if n == 0:
        return a
    delta = mb - ma
    mean = ma + delta * nb / n
    m2 = qa + qb + delta * delta * na * nb / n
    return n, mean, m2, min(mna, mnb), max(mxa, mxb)


def moments(x: torch.Tensor, group=None, ddof: int = 0) -> dict:
    if x.dtype not in (torch.float32, torch.float64, torch.bfloat16, torch.float16):
        raise TypeError("moments: float32, float64, bfloat16 or float16 input")
    x = x.contiguous().reshape(-1)
    r = _raw(x)
    if group is not None or (torch.distributed.is_initialized() and torch.distributed.get_world_size() > 1):
        world = torch.distributed.get_world_size(group)
        mine = torch.tensor([float(v) for v in r], dtype=torch.float64,
                            device=x.device if torch.distributed.get_backend(group) == "nccl" else "cpu")
        allv = [torch.empty_like(mine) for _ in range(world)]
        torch.distributed.all_gather(allv, mine, group=group)
        acc = (0, 0.0, 0.0, math.inf, -math.inf)
        for t in allv:
            v = t.tolist()
            acc = combine_moments(acc, (int(v[0]), v[1], v[2], v[3], v[4]))
        r = acc
    n, mean, m2, mn, mx = r
    var = m2 / (n - ddof) if n - ddof > 0 else float("nan")
    return {"count": n, "sum": mean * n, "mean": mean, "var": var, "std": math.sqrt(var) if var == var else var,
            "min": mn, "max": mx}
