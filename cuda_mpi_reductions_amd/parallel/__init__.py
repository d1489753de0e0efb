"""Distributed layer: one process per GPU, RCCL (torch backend "nccl") over xGMI."""
from .dist import (  # noqa: F401
    DistContext, barrier, init, max_over_ranks, reduce_op, scalar_allreduce, shard, shutdown,
    vector_allreduce, vector_reduce,
)
