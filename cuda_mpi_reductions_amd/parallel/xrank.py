"""Fused cross-rank finish: the scalar all-reduce folded into the reduction kernel itself.

The hybrid "local reduce, then reduce one value across ranks" of the vendored simpleMPI
(cuda/C/src/simpleMPI/simpleMPI.cpp:92-98; SURVEY.md §5.8 mode scalar) normally costs a second
collective launch (RCCL all-reduce of 1 element) on its own stream. With an :class:`XrankChannel`
bound to the reduction (``Reducer.bind(..., xrank=channel)``) the kernel's last workgroup pushes
its partial into every rank's mailbox over xGMI and folds the ranks' partials itself
(csrc/include/mireduce/xrank.hpp): one kernel per global reduction, graph-capturable, the result
bit-identical on every rank.

:func:`open_channel` is collective over the default process group (or ``group``): every rank
allocates a mailbox, the IPC handles are all-gathered, every peer's mailbox is mapped.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .._native import native

__all__ = ["open_channel", "check_channel"]


def open_channel(device: torch.device, group=None, timeout_s: float = 2.0):
    """Create and connect this rank's :class:`_C.XrankChannel` (collective)."""
    C = native()
    idx = device.index if device.index is not None else torch.cuda.current_device()
    ch = C.XrankChannel(idx, timeout_s)
    if dist.is_available() and dist.is_initialized():
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        if world > C.XRANK_MAX_RANKS:
            raise ValueError(f"fused finish supports at most {C.XRANK_MAX_RANKS} ranks, got {world}")
        handles: list = [None] * world
        dist.all_gather_object(handles, ch.handle(), group=group)
    else:
        rank, world, handles = 0, 1, [ch.handle()]
    ch.connect(rank, world, handles)
    if world > 1:
        dist.barrier(group=group)  # every rank mapped every mailbox before anyone pushes
    return ch


def check_channel(channels, group=None) -> Optional[str]:
    """None if no channel's kernel ever timed out on any rank, else an error string (collective
    when a process group is initialised: every rank gets the same verdict)."""
    bad = sum(int(ch.error()) for ch in channels)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = torch.tensor([bad], dtype=torch.int64)
        if dist.get_backend(group) == "nccl":
            t = t.cuda()
        dist.all_reduce(t, group=group)
        bad = int(t.item())
    return None if bad == 0 else f"fused cross-rank finish: {bad} channel(s) timed out waiting for a peer"
