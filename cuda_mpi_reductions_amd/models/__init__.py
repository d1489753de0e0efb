"""Benchmark workloads (the BASELINE.json configs)."""
from .workloads import (  # noqa: F401
    COLLECTIVES, CONFIGS, NORTH_STAR, ScalarReduction, VectorReduction, WorkloadConfig, element_size,
)
from .loc import LOC_OPS, LocReduction  # noqa: F401


def scalar_workload(cfg, ctx, kernel=None, streams: int = 1, collective: str = "rccl",
                    always_collective: bool = False, xrank_timeout_s: float = 10.0, fault=None):
    """The array -> one-result workload of a scalar-mode config: MAXLOC/MINLOC configs get
    :class:`LocReduction` (RCCL combine only), every other operator :class:`ScalarReduction`."""
    if cfg.op in LOC_OPS:
        if collective != "rccl":
            raise ValueError("MAXLOC/MINLOC configs combine over RCCL only (--collective rccl)")
        return LocReduction(cfg, ctx, kernel, always_collective=always_collective)
    return ScalarReduction(cfg, ctx, kernel, streams=streams, collective=collective,
                           always_collective=always_collective, xrank_timeout_s=xrank_timeout_s, fault=fault)
