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
from .topology import peer_map

__all__ = ["open_channel", "check_channel", "close_channels"]


def open_channel(device: torch.device, group=None, timeout_s: float = 2.0, fault=None):
    """Create and connect this rank's :class:`_C.XrankChannel` (collective). ``fault`` (a
    :class:`utils.fault.FaultInjector`, kind ``mailbox``) makes one rank fail to create its mailbox:
    the failure-path test of the collective agreement below."""
    C = native()
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if not (dist.is_available() and dist.is_initialized()):
        ch = C.XrankChannel(idx, timeout_s)
        ch.connect(0, 1, [ch.handle()])
        return ch
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world > C.XRANK_MAX_RANKS:
        raise ValueError(f"fused finish supports at most {C.XRANK_MAX_RANKS} ranks, got {world}")
    pm = peer_map(idx, group)  # collective; the same verdict on every rank
    if pm.error:
        raise RuntimeError("fused cross-rank finish unavailable: " + pm.error)
    # Every step below is reached by every rank (errors are agreed on, not raised mid-protocol),
    # so one rank's failure to allocate or map cannot leave the others blocked in a collective.
    err, ch, handle = None, None, b""
    try:
        if fault is not None and fault.mailbox(rank):
            raise RuntimeError("injected mailbox failure (--inject-fault mailbox)")
        ch = C.XrankChannel(idx, timeout_s)
        handle = ch.handle()
    except Exception as e:  # noqa: BLE001 - reported collectively below
        err = f"{type(e).__name__}: {e}"
    handles: list = [None] * world
    dist.all_gather_object(handles, handle, group=group)
    if err is None:
        if any(not h for h in handles):
            err = "a peer could not create its mailbox"
        else:
            try:
                ch.connect(rank, world, handles)
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
    errs: list = [None] * world
    dist.all_gather_object(errs, err, group=group)  # also the barrier: all mailboxes mapped
    # the ranks that failed themselves first (the others only saw a missing peer)
    own = [f"rank {r}: {m}" for r, m in enumerate(errs) if m and not m.startswith("a peer")]
    bad = own + [f"rank {r}: {m}" for r, m in enumerate(errs) if m and m.startswith("a peer")]
    if bad:
        raise RuntimeError("fused cross-rank finish unavailable: " + "; ".join(bad)[:500])
    return ch


def check_channel(channels, group=None) -> Optional[str]:
    """None if no channel's kernel ever flagged an error on any rank (a peer's partial late, or
    poisoned by that peer's failed fan-in), else an error string (collective when a process group
    is initialised: every rank gets the same verdict)."""
    bad = sum(int(ch.error() != 0) for ch in channels)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        t = torch.tensor([bad], dtype=torch.int64)
        if dist.get_backend(group) == "nccl":
            t = t.cuda()
        dist.all_reduce(t, group=group)
        bad = int(t.item())
    return None if bad == 0 else (f"fused cross-rank finish: {bad} channel(s) flagged an error (a peer's "
                                  "partial timed out or arrived poisoned)")


def close_channels(channels: list, device: torch.device, group=None) -> None:
    """Collective teardown of this rank's channels (the caller drops every other reference, e.g.
    the bound reductions, first): the list is emptied, mappings closed, mailboxes freed, then all
    ranks meet — a channel opened next may reuse a mailbox address, and its IPC export must not
    race a peer that still maps the old mailbox there."""
    had = bool(channels)
    if had:
        torch.cuda.synchronize(device)
    channels.clear()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if dist.get_backend(group) == "nccl":
            dist.barrier(group=group, device_ids=[device.index])
        else:
            dist.barrier(group=group)
