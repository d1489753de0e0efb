"""Distributed layer: one process per GPU, RCCL (torch backend "nccl") over xGMI."""
from .dist import (  # noqa: F401
    DistContext, barrier, init, max_over_ranks, reduce_op, scalar_allreduce, shard, shutdown,
    vector_allreduce, vector_reduce,
)
from .direct import DirectComm  # noqa: F401,E402
from .topology import PeerMap, peer_map, peer_verdict  # noqa: F401,E402
from .xrank import check_channel, open_channel  # noqa: F401,E402
