"""cuda_mpi_reductions_amd (``mireduce``) — an MI355X-native parallel-reduction framework.

Capability parity target: ``szabodabo/CUDA-MPI-Reductions`` — single-GPU SUM/MIN/MAX tree
reductions (cuda/C/src/reduction/) and cross-rank ``MPI_Reduce`` benchmarks (mpi/reduce.c) —
re-designed for gfx950: hand-written HIP streaming kernels (csrc/kernels/reduce.hip), RCCL over
xGMI through ``torch.distributed`` (backend "nccl") and a native C++ RCCL/MPI runtime
(csrc/comm, csrc/apps).

Layout:
    ops/       tensor-level reductions and fills backed by the HIP kernels
    parallel/  process-group setup, sharding, scalar / vector cross-rank reductions
    models/    benchmark workloads (the BASELINE.json configs) — the "models" of this framework
    utils/     reference-compatible CLI grammar, output formats, averaging, timers, QA lines
"""
from ._native import available as native_available  # noqa: F401

__version__ = "0.1.0"

from . import ops, parallel, models, utils  # noqa: E402,F401
