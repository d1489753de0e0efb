"""Who shares a GPU with whom, and can every rank's GPU map every peer's memory?

The two IPC-mapped xGMI paths — the fused cross-rank finish (:mod:`.xrank`) and the direct
collective (:mod:`.direct`) — store into / load from peers' device memory from inside a kernel.
That needs every rank on one host (HIP IPC handles do not cross nodes) and peer access between every
pair of distinct devices (the vendored simpleP2P checks the same with ``cudaDeviceCanAccessPeer``
before it maps anything, cuda/C/src/simpleP2P/simpleP2P.cu:250-275). A rank that went ahead
without it would fault the GPU instead of failing a host call, so both paths ask
:func:`peer_map` first and decline on every rank together when it says no.

Ranks sharing one physical GPU (the one-GPU rehearsals) need no peer access between them, and the
direct collective divides the GPU's CUs among them (``ranks_per_gpu``).
"""
from __future__ import annotations

import socket
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

__all__ = ["PeerMap", "peer_map", "peer_verdict", "forget"]

Key = Tuple[str, str, int]  # (host, device uuid or PCI id, local device index)


@dataclass(frozen=True)
class PeerMap:
    keys: Tuple[Key, ...]      # one per rank, in rank order
    ranks_per_gpu: int         # the most ranks on one physical GPU
    error: Optional[str]       # None: every rank can map every peer's memory


def peer_verdict(keys: Sequence[Key], me: int, can_access: Callable[[int, int], bool]) -> Optional[str]:
    """This rank's verdict (pure; ``can_access(my_index, peer_index)``): None, or why rank ``me``
    cannot map some peer's memory."""
    host, uuid, idx = keys[me]
    for r, (h, u, d) in enumerate(keys):
        if r == me or u == uuid and h == host:
            continue  # itself, or a rank on the same physical GPU
        if h != host:
            return f"rank {r} runs on host {h}, not {host} (IPC handles do not cross hosts)"
        if d == idx:
            return f"rank {r} reports device {d} = mine but a different GPU ({u} vs {uuid})"
        if not can_access(idx, d):
            return f"device {idx} cannot access peer device {d} (rank {r})"
    return None


def _key(idx: int) -> Key:
    props = torch.cuda.get_device_properties(idx)
    return (socket.gethostname(), str(getattr(props, "uuid", "")) or str(getattr(props, "pci_bus_id", idx)), idx)


# Answers per (group object, device). The group object itself is held (not its id(), which a later
# group could reuse on some ranks only: those would skip the gathers the others enter and the job
# would hang); forget() — called by parallel.dist.shutdown — drops them with the groups.
_cache: list = []


def forget() -> None:
    """Drop every remembered answer (process groups are being destroyed)."""
    _cache.clear()


def peer_map(idx: int, group=None) -> PeerMap:
    """Collective over ``group``: every rank's (host, GPU, index), and one verdict agreed by all
    ranks (every rank gets the same ``error``). Remembered per (group, device): every rank asks
    with the same arguments, so every rank takes the cached answer together. A rank whose own
    (host, GPU) query fails still enters both gathers (with the failure as its key), so the
    verdict is an error on every rank instead of a hang on the others."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return PeerMap((_key(idx),), 1, None)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    for g, i, w, r, pm in _cache:
        if g is pg and (i, w, r) == (idx, world, rank):
            return pm
    try:
        key = _key(idx)
    except Exception as e:  # noqa: BLE001 - agreed on below, never raised mid-protocol
        key = ("?", f"unknown ({type(e).__name__}: {e})"[:200], idx)
        mine = f"cannot query device {idx}: {type(e).__name__}: {e}"
    else:
        mine = None
    keys: List = [None] * world
    dist.all_gather_object(keys, key, group=group)
    keys = [tuple(k) for k in keys]
    if mine is None:
        try:
            mine = peer_verdict(keys, rank, torch.cuda.can_device_access_peer)
        except Exception as e:  # noqa: BLE001 - agreed on below, never raised mid-protocol
            mine = f"{type(e).__name__}: {e}"
    verdicts: List = [None] * world
    dist.all_gather_object(verdicts, mine, group=group)
    bad = [f"rank {r}: {m}" for r, m in enumerate(verdicts) if m]
    gpus = [(h, u) for h, u, _ in keys]
    pm = PeerMap(tuple(keys), max(gpus.count(g) for g in gpus), "; ".join(bad)[:500] if bad else None)
    _cache.append((pg, idx, world, rank, pm))
    return pm
