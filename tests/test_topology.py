"""Peer-map preflight of the IPC-mapped xGMI paths (parallel/topology.py): the per-rank verdict
(pure) and the collective agreement over gloo, with the device queries stubbed (CPU-only box)."""
import os

import torch.multiprocessing as mp

from helpers import free_port

from cuda_mpi_reductions_amd.parallel.topology import peer_verdict

ALL = lambda a, b: True  # noqa: E731


def _node(n, host="h0"):
    return [(host, f"gpu{i}", i) for i in range(n)]


def test_one_node_all_peers_mapped():
    keys = _node(8)
    assert all(peer_verdict(keys, r, ALL) is None for r in range(8))


def test_ranks_sharing_one_gpu_need_no_peer_access():
    keys = [("h0", "gpu0", 0)] * 4
    assert peer_verdict(keys, 2, lambda a, b: False) is None


def test_missing_peer_access_declines():
    keys = _node(4)
    v = peer_verdict(keys, 1, lambda a, b: not (a == 1 and b == 3))
    assert v is not None and "device 1 cannot access peer device 3" in v
    assert peer_verdict(keys, 0, lambda a, b: not (a == 1 and b == 3)) is None


def test_other_host_declines():
    keys = _node(2) + _node(2, host="h1")
    assert "IPC handles do not cross hosts" in peer_verdict(keys, 0, ALL)


def test_same_index_other_gpu_declines():
    # per-rank device masks: every rank sees its own GPU as device 0
    keys = [("h0", "gpuA", 0), ("h0", "gpuB", 0)]
    assert "different GPU" in peer_verdict(keys, 0, ALL)


def _worker(rank, world, port, deny_rank, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import torch
        import torch.distributed as dist
        from cuda_mpi_reductions_amd.parallel import topology
        topology._key = lambda idx: ("h0", f"gpu{rank}", rank)  # one GPU per rank, one host
        torch.cuda.can_device_access_peer = lambda a, b: a != deny_rank
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pm = topology.peer_map(rank)
        again = topology.peer_map(rank)  # cached: no collective, same answer
        dist.destroy_process_group()
        q.put((rank, (pm.error, pm.ranks_per_gpu, again is pm)))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def _run(world, deny_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, deny_rank, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    return out


def test_peer_map_agreed_by_every_rank():
    ok = _run(3, deny_rank=-1)
    assert all(v == (None, 1, True) for v in ok.values()), ok
    bad = _run(3, deny_rank=2)
    errs = {v[0] for v in bad.values()}
    assert len(errs) == 1, bad  # the same verdict on every rank
    (err,) = errs
    assert err.startswith("rank 2: device 2 cannot access peer device 0"), err
