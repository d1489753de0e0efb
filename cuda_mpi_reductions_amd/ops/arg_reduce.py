"""Arg-reductions: ``arg_reduce(x, "max" | "min", dim)`` -> ``(values, indices)`` ~ ``torch.max/min(x, dim)``.

Not in the reference, whose MIN/MAX return the extreme value only
(cuda/C/src/reduction/reduction_kernel.cu:128-253; mpi/reduce.c:21-28); the position of the
extreme is the other thing a reduction framework is asked for (greedy decoding over a vocabulary,
top-1 routing over experts, locating the worst element of a residual). Semantics are torch's:
the FIRST index of the extreme, NaN counts as the extreme (the first NaN wins), -0.0 == +0.0.

Device tensors run csrc/kernels/arg_reduce.hip (one launch; whole arrays and long rows are split
into segments streamed by whole workgroups and finished single-pass by the last arriving segment;
short rows use lane groups). Host tensors run the native host reference (same semantics).
``dim`` other than the last axis is moved last first (one copy). With ``group`` (``dim=None``),
the result is the global first extreme over every rank's shard, indexed in the concatenation of
the shards in rank order.
"""
from __future__ import annotations

import threading
from typing import Optional, Tuple

import torch

from .._native import native
from .reduce import DTYPE_CODES, op_code

__all__ = ["arg_reduce", "argmax", "argmin"]

_scratch: dict = {}
_lock = threading.Lock()


def _zeroed_scratch(device: torch.device, nbytes: int) -> torch.Tensor:
    """Per-(device, stream) zero-initialised scratch; the kernel leaves its ticket words zero."""
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    with _lock:
        buf = _scratch.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.zeros(max(nbytes, 1 << 16), dtype=torch.uint8, device=device)
            _scratch[key] = buf
        return buf


def _rows(x2: torch.Tensor, op: str) -> Tuple[torch.Tensor, torch.Tensor]:
    """(values, indices) of every row of a contiguous 2-D tensor."""
    if x2.dtype not in DTYPE_CODES:
        raise TypeError(f"arg_reduce: unsupported dtype {x2.dtype}")
    rows, cols = x2.shape
    if cols == 0:
        raise ValueError("arg_reduce over an empty dimension")
    vals = torch.empty(rows, dtype=x2.dtype, device=x2.device)
    idx = torch.empty(rows, dtype=torch.int64, device=x2.device)
    if rows == 0:
        return vals, idx
    C = native()
    dt, oc = DTYPE_CODES[x2.dtype], op_code(op)
    if x2.device.type != "cuda":
        C.cpu_arg_reduce_rows(x2.data_ptr(), rows, cols, dt, oc, vals.data_ptr(), idx.data_ptr())
        return vals, idx
    ncu = torch.cuda.get_device_properties(x2.device).multi_processor_count
    need = C.arg_reduce_scratch_bytes(rows, cols, dt, ncu)
    scratch = _zeroed_scratch(x2.device, need) if need else None
    C.arg_reduce_rows(x2.data_ptr(), rows, cols, dt, oc, vals.data_ptr(), idx.data_ptr(),
                      scratch.data_ptr() if scratch is not None else 0, ncu,
                      torch.cuda.current_stream(x2.device).cuda_stream)
    return vals, idx


def arg_reduce(x: torch.Tensor, op: str = "max", dim: Optional[int] = None, keepdim: bool = False,
               group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """``(values, indices)`` of the first maximum (``op="max"``) or minimum (``op="min"``).

    ``dim=None`` reduces the whole (flattened) tensor to 0-d results; otherwise along ``dim``.
    ``group`` (``dim=None`` only): reduce over all ranks' shards of one logical array (pass
    ``torch.distributed.group.WORLD`` for the default group); without it the call is rank-local.
    """
    op = op.lower()
    if op not in ("max", "min"):
        raise ValueError("arg_reduce: op must be 'max' or 'min'")
    if dim is None:
        if x.numel() == 0:
            raise ValueError("arg_reduce of an empty tensor")
        v, i = _rows(x.contiguous().view(1, -1), op)
        v, i = v.reshape(()), i.reshape(())
        if group is not None:  # global only when asked: a rank-local call must stay local
            v, i = _global(v, i, x.numel(), op, group)
        if keepdim:
            shape = [1] * x.dim()
            return v.reshape(shape), i.reshape(shape)
        return v, i
    if group is not None:
        raise ValueError("arg_reduce: group is supported for dim=None only")
    if x.dim() == 0:
        raise ValueError("arg_reduce along a dimension needs at least one dimension")
    dim = dim % x.dim()
    xm = x if dim == x.dim() - 1 else x.movedim(dim, -1)
    lead = list(xm.shape[:-1])
    v, i = _rows(xm.contiguous().view(-1, xm.shape[-1]), op)
    v, i = v.view(lead), i.view(lead)
    if keepdim:
        v, i = v.unsqueeze(dim), i.unsqueeze(dim)
    return v, i


def argmax(x: torch.Tensor, dim: Optional[int] = None, keepdim: bool = False) -> torch.Tensor:
    """First index of the maximum (``torch.argmax`` semantics)."""
    return arg_reduce(x, "max", dim, keepdim)[1]


def argmin(x: torch.Tensor, dim: Optional[int] = None, keepdim: bool = False) -> torch.Tensor:
    """First index of the minimum (``torch.argmin`` semantics)."""
    return arg_reduce(x, "min", dim, keepdim)[1]


def _global(v: torch.Tensor, i: torch.Tensor, local_n: int, op: str, group):
    """Global first extreme over the ranks' shards (concatenated in rank order): all-gather every
    rank's (value, local index, shard length), then arg-reduce the gathered values — ranks are in
    order, so the first-occurrence rule carries over."""
    d = torch.distributed
    world = d.get_world_size(group)
    host = d.get_backend(group) == "gloo" or v.device.type == "cpu"
    dev = torch.device("cpu") if host else v.device
    meta = torch.stack([i.to(torch.int64), torch.tensor(local_n, dtype=torch.int64, device=i.device)]).to(dev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    vals = [torch.empty_like(v.to(dev).reshape(1)) for _ in range(world)]
    d.all_gather(metas, meta, group=group)
    d.all_gather(vals, v.to(dev).reshape(1), group=group)
    allv = torch.cat(vals).cpu()
    winner = int(_rows(allv.view(1, -1), op)[1][0])
    lens = [int(m[1]) for m in metas]
    gidx = sum(lens[:winner]) + int(metas[winner][0])
    return allv[winner].to(v.device).reshape(()), torch.tensor(gidx, dtype=torch.int64, device=i.device)
