"""Reductions along one dimension: ``reduce_dim(x, op, dim)`` ~ ``torch.sum/amin/amax(x, dim)``.

Not in the reference (its reductions collapse whole arrays: cuda/C/src/reduction/reduction.cpp:
661-1034; mpi/reduce.c:76,90), but the per-axis form is the other half of what a reduction
framework on MI355X is asked for. Device tensors run csrc/kernels/reduce_dim.hip:

* ``dim`` is the last (contiguous) axis -> row mode: wave-granular row segments, 16-byte nt loads,
  split rows finished single-pass by the last arriving segment;
* ``dim`` is the first axis of a contiguous tensor -> column mode: 16 bytes of adjacent columns per
  thread walking down the rows, row ranges folded by a second launch when columns are few;
* any other axis: the tensor is viewed as ``[outer, D, inner]`` and the column kernel runs over
  all ``outer`` slabs in one launch (grid.z; no copy).

Host tensors fall back to torch (the dimension forms have no reference counterpart to match).
Accumulator defaults follow :func:`default_acc_dtype` (int32 SUM -> int64, fp32 SUM -> fp64,
bf16/fp16 -> fp32).
"""
from __future__ import annotations

import threading
from typing import Optional

import torch

from .._native import native
from .reduce import default_acc_dtype, dtype_code, op_code

__all__ = ["reduce_dim"]

_scratch: dict = {}
_lock = threading.Lock()


def _zeroed_scratch(device: torch.device, nbytes: int, kind: str) -> torch.Tensor:
    """Per-(device, stream, kind) zero-initialised scratch. Row mode's ticket words must be zero on
    entry (its kernels leave them zero); column mode writes partials, so the two never share."""
    key = (device.index, torch.cuda.current_stream(device).cuda_stream, kind)
    with _lock:
        buf = _scratch.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.zeros(max(nbytes, 1 << 16), dtype=torch.uint8, device=device)
            _scratch[key] = buf
        return buf


def _num_cus(device: torch.device) -> int:
    return torch.cuda.get_device_properties(device).multi_processor_count


def reduce_dim(x: torch.Tensor, op: str = "sum", dim: int = -1, acc_dtype: Optional[torch.dtype] = None,
               keepdim: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Reduce ``x`` along ``dim`` with ``op`` in {"sum", "min", "max"}; result dtype = accumulator."""
    if x.dim() == 0:
        raise ValueError("reduce_dim needs at least one dimension")
    dim = dim % x.dim()
    acc = acc_dtype or default_acc_dtype(x.dtype, op)
    shape = list(x.shape)
    out_shape = shape[:dim] + ([1] if keepdim else []) + shape[dim + 1:]
    if x.device.type != "cuda":
        fn = {"sum": lambda t: t.sum(dim=dim, keepdim=keepdim, dtype=acc),
              "min": lambda t: t.amin(dim=dim, keepdim=keepdim).to(acc),
              "max": lambda t: t.amax(dim=dim, keepdim=keepdim).to(acc)}[op.lower()]
        res = fn(x.to(acc) if op.lower() != "sum" else x)
        if out is not None:
            out.copy_(res)
            return out
        return res
    if shape[dim] == 0:
        raise ValueError("reduce_dim over an empty dimension")
    C = native()
    x = x.contiguous()
    outer = 1
    for s in shape[:dim]:
        outer *= s
    inner = 1
    for s in shape[dim + 1:]:
        inner *= s
    d = shape[dim]
    if out is None:
        out = torch.empty(out_shape, dtype=acc, device=x.device)
    elif out.dtype != acc or not out.is_contiguous() or out.numel() != outer * inner:
        raise ValueError("out must be a contiguous tensor of the accumulator dtype with the reduced shape")
    if out.numel() == 0:
        return out
    stream = torch.cuda.current_stream(x.device).cuda_stream
    ncu = _num_cus(x.device)
    dt, oc, ac = dtype_code(x.dtype), op_code(op), dtype_code(acc)
    if inner == 1:  # contiguous axis: one row per output element
        need = C.reduce_rows_scratch_bytes(outer, d, dt, ncu)
        scratch = _zeroed_scratch(x.device, need, "rows") if need else None
        C.reduce_rows(x.data_ptr(), outer, d, dt, oc, ac, out.data_ptr(),
                      scratch.data_ptr() if scratch is not None else 0, ncu, stream)
        return out
    need = C.reduce_cols_scratch_bytes(outer, d, inner, dt, ac, ncu)
    scratch = _zeroed_scratch(x.device, need, "cols") if need else None
    C.reduce_cols(x.data_ptr(), outer, d, inner, dt, oc, ac, out.data_ptr(),
                  scratch.data_ptr() if scratch is not None else 0, ncu, stream)
    return out
