"""Synthetic data generation (device fill + bit-identical host fill).

Reference data: ``rand() & 0xFF`` in the CUDA sample (cuda/C/src/reduction/reduction.cpp:698-705)
and MT19937 in the MPI benchmark (mpi/reduce.c:38-57). Element ``i`` is a pure function of
``(seed, offset + i)`` (csrc/include/mireduce/rng.hpp), so a sharded array filled on N GPUs is the
same logical array for every N and any element can be recomputed on the host.
"""
from __future__ import annotations

import torch

from .._native import native
from .reduce import dtype_code

PATTERNS = {"uniform": 0, "smallint": 1, "fullrange": 2, "iotamod": 3, "constant": 4}

__all__ = ["PATTERNS", "fill_", "synthetic", "mt19937_fill_"]


def pattern_code(p: str) -> int:
    try:
        return PATTERNS[p.lower()]
    except KeyError:
        raise ValueError(f"unknown pattern {p!r}; choose from {sorted(PATTERNS)}") from None


def fill_(x: torch.Tensor, pattern: str = "uniform", seed: int = 0x5EED, offset: int = 0,
          value: float = 0.0) -> torch.Tensor:
    """Fill ``x`` in place. Device tensors use the HIP fill kernel on the current stream."""
    C = native()
    if not x.is_contiguous():
        raise ValueError("fill_ needs a contiguous tensor")
    if x.device.type == "cuda":
        stream = torch.cuda.current_stream(x.device).cuda_stream
        C.fill_device(x.data_ptr(), x.numel(), dtype_code(x.dtype), pattern_code(pattern), seed, offset,
                      float(value), stream)
    else:
        C.fill_host(x.data_ptr(), x.numel(), dtype_code(x.dtype), pattern_code(pattern), seed, offset,
                    float(value))
    return x


def synthetic(n: int, dtype: torch.dtype, device="cpu", pattern: str = "uniform", seed: int = 0x5EED,
              offset: int = 0, value: float = 0.0) -> torch.Tensor:
    x = torch.empty(n, dtype=dtype, device=device)
    return fill_(x, pattern, seed, offset, value)


def mt19937_fill_(x: torch.Tensor, rank: int) -> torch.Tensor:
    """reduce.c's per-rank data: seeds {rank,0x123,0x234,0x345,0x456,0x789} (mpi/reduce.c:38-41);
    int32 from genrand_int32 (wrapping cast), float64 from genrand_res53 (mpi/reduce.c:51-57)."""
    C = native()
    if x.device.type != "cpu" or not x.is_contiguous():
        raise ValueError("mt19937_fill_ needs a contiguous host tensor")
    g = C.Mt19937()
    g.init_by_array([rank, 0x123, 0x234, 0x345, 0x456, 0x789])
    if x.dtype == torch.int32:
        g.fill_int32(x.data_ptr(), x.numel())
    elif x.dtype == torch.float64:
        g.fill_res53(x.data_ptr(), x.numel())
    else:
        raise TypeError("reduce.c generates int32 and float64 only")
    return x
