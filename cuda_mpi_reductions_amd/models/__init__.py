"""Benchmark workloads (the BASELINE.json configs)."""
from .workloads import (  # noqa: F401
    CONFIGS, NORTH_STAR, ScalarReduction, VectorReduction, WorkloadConfig, element_size,
)
from .loc import LOC_OPS, LocReduction  # noqa: F401


def scalar_workload(cfg, ctx, kernel=None, streams: int = 1):
    """The array -> one-result workload of a scalar-mode config: MAXLOC/MINLOC configs get
    :class:`LocReduction`, every other operator :class:`ScalarReduction`."""
    if cfg.op in LOC_OPS:
        return LocReduction(cfg, ctx, kernel)
    return ScalarReduction(cfg, ctx, kernel, streams=streams)
