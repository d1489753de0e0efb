"""Global norms of (sharded) tensors: the fused SUMSQ / AMAX kernels plus the reference's hybrid
pattern — local GPU reduce, then a scalar cross-rank reduction (cuda/C/src/simpleMPI/
simpleMPI.cpp:92-98).

``norm(x, 2)`` = sqrt(Σ x²) with the square fused into the streaming load (one pass over HBM, no
``x * x`` temporary); ``norm(x, inf)`` = max |x| (the amax that FP8 scaling factors are computed
from). With a process group (or an initialised multi-rank default group) each rank passes its
shard and every rank gets the norm of the whole distributed tensor.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from .reduce import reduce

__all__ = ["norm"]


def norm(x: torch.Tensor, p: float = 2, group=None, acc_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """L2 (``p=2``) or max (``p=inf``) norm of ``x`` — of all ranks' shards when distributed.
    Returns a 1-element tensor of the accumulator dtype (fp64 for fp32/fp64 L2, fp32 for bf16/fp16)."""
    if not x.dtype.is_floating_point:
        raise TypeError("norm needs a floating-point tensor")
    if p == 2:
        op = "sumsq"
    elif p == math.inf or p == "inf":
        op = "amax"
    else:
        raise ValueError("norm: p must be 2 or inf")
    r = reduce(x.reshape(-1), op, acc_dtype)
    dist = torch.distributed
    if group is not None or (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        rop = dist.ReduceOp.SUM if op == "sumsq" else dist.ReduceOp.MAX
        if dist.get_backend(group) == "gloo" and r.device.type != "cpu":
            h = r.cpu()
            dist.all_reduce(h, op=rop, group=group)
            r.copy_(h)
        else:
            dist.all_reduce(r, op=rop, group=group)
    return r.sqrt_() if op == "sumsq" else r
