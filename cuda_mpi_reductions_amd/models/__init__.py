"""Benchmark workloads (the BASELINE.json configs)."""
from .workloads import (  # noqa: F401
    CONFIGS, NORTH_STAR, ScalarReduction, VectorReduction, WorkloadConfig, element_size,
)
