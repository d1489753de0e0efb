"""One launch over a list of tensors: ``reduce_many([t0, t1, ...], op)`` -> ``[op(t0), op(t1), ...]``.

The multi-tensor form of the full reduction (csrc/kernels/reduce_many.hip): every tensor of the
list is cut into segments that the waves of ONE kernel share, so a list of many small tensors
costs one launch and one tail instead of one per tensor. ``ReduceMany`` binds a fixed list once
(segment table uploaded to the GPU) and ``__call__`` is then a single, graph-capturable launch —
the per-step shape of e.g. gradient-norm clipping over a model's parameter shards.
``norm_many`` adds the total norm over the list and, when distributed, over all ranks' shards
(the reference's local-reduce + scalar cross-rank step, cuda/C/src/simpleMPI/simpleMPI.cpp:92-98).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Optional, Sequence

import torch

from .._native import native
from .reduce import default_acc_dtype, dtype_code, op_code

__all__ = ["ReduceMany", "reduce_many", "norm_many"]


class ReduceMany:
    """A bound list: ``rm()`` enqueues one launch writing ``rm.out[i] = op(tensors[i])``. The tensors
    must stay alive (and keep their storage) while this object is used."""

    def __init__(self, tensors: Sequence[torch.Tensor], op: str = "sum", acc_dtype: Optional[torch.dtype] = None):
        if not tensors:
            raise ValueError("reduce_many: empty tensor list")
        dev, dt = tensors[0].device, tensors[0].dtype
        for t in tensors:
            if t.device != dev or t.dtype != dt:
                raise ValueError("reduce_many: all tensors must share device and dtype (group them first)")
            if not t.is_contiguous():
                raise ValueError("reduce_many: tensors must be contiguous")
        if dev.type != "cuda":
            raise ValueError("reduce_many: device tensors only (host tensors: use reduce per tensor)")
        self.tensors = list(tensors)
        self.op = op
        self.acc = acc_dtype or default_acc_dtype(dt, op)
        self.out = torch.empty(len(tensors), dtype=self.acc, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        self._b = native().BoundReduceMany([t.data_ptr() for t in tensors], [t.numel() for t in tensors],
                                           dtype_code(dt), op_code(op), dtype_code(self.acc), self.out.data_ptr(),
                                           dev.index if dev.index is not None else torch.cuda.current_device(),
                                           ncu, stream)
        self.device = dev

    @property
    def segments(self) -> int:
        return self._b.segments

    def __call__(self, stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        self._b.launch(s.cuda_stream)
        return self.out


_bindings: "OrderedDict[tuple, ReduceMany]" = OrderedDict()
_MAX_BINDINGS = 32


def _binding(tensors: Sequence[torch.Tensor], op: str, acc_dtype) -> ReduceMany:
    """A cached :class:`ReduceMany` for this exact list (pointers, sizes, dtype, op, stream): repeated
    calls on the same parameters (a per-step grad norm) reuse its device table — no allocation,
    upload or synchronisation per call. Evicted bindings are freed after their stream drains."""
    dev = tensors[0].device
    stream = torch.cuda.current_stream(dev)
    key = (dev.index, stream.cuda_stream, tensors[0].dtype, op, acc_dtype,
           tuple(t.data_ptr() for t in tensors), tuple(t.numel() for t in tensors))
    rm = _bindings.get(key)
    if rm is not None:
        _bindings.move_to_end(key)
        return rm
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("reduce_many: first call for this tensor list inside a graph capture; call it once "
                           "before capturing (or capture a ReduceMany object built beforehand)")
    rm = ReduceMany(list(tensors), op, acc_dtype)
    _bindings[key] = rm
    while len(_bindings) > _MAX_BINDINGS:
        _, old = _bindings.popitem(last=False)
        stream.synchronize()  # launches of the evicted binding may still be in flight
        del old
    return rm


def reduce_many(tensors: Sequence[torch.Tensor], op: str = "sum", acc_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """Per-tensor reduction of a list in one launch (device tensors); host lists fall back to the
    native host reducer per tensor. Returns a fresh tensor each call (the binding is cached)."""
    if tensors and tensors[0].device.type != "cuda":
        from .reduce import reduce
        acc = acc_dtype or default_acc_dtype(tensors[0].dtype, op)
        return torch.cat([reduce(t.reshape(-1), op, acc) for t in tensors])
    tensors = [t.contiguous() for t in tensors]
    if any(not t.is_contiguous() for t in tensors):  # pragma: no cover
        raise ValueError("reduce_many needs contiguous tensors")
    rm = _binding(tensors, op, acc_dtype)
    out = torch.empty_like(rm.out)
    rm._b.launch(torch.cuda.current_stream(rm.device).cuda_stream, out.data_ptr())
    return out


def norm_many(tensors: Sequence[torch.Tensor], p: float = 2, group=None):
    """(total norm, per-tensor norms) of a list of floating tensors — L2 (``p=2``) or max (``p=inf``)
    — with the total taken over every rank's list when distributed."""
    if p == 2:
        op = "sumsq"
    elif p == math.inf or p == "inf":
        op = "amax"
    else:
        raise ValueError("norm_many: p must be 2 or inf")
    per = reduce_many(tensors, op)
    total = (per.sum() if op == "sumsq" else per.max()).reshape(1)
    dist = torch.distributed
    if group is not None or (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        rop = dist.ReduceOp.SUM if op == "sumsq" else dist.ReduceOp.MAX
        if dist.get_backend(group) == "gloo" and total.device.type != "cpu":
            h = total.cpu()
            dist.all_reduce(h, op=rop, group=group)
            total.copy_(h)
        else:
            dist.all_reduce(total, op=rop, group=group)
    if op == "sumsq":
        return total.sqrt_(), per.sqrt()
    return total, per
