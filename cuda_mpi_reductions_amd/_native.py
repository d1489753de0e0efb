"""Loader for the native extension ``cuda_mpi_reductions_amd._C`` (built by ``make python``).

The HIP kernels live only in the native extension; there is deliberately no PyTorch fallback for
device tensors. If the extension is missing the import error is raised loudly (on a GPU box a
silent eager fallback would hide that the native path did not run).
"""
from __future__ import annotations

import importlib
import os

# torch must be imported BEFORE the extension: torch ships its own libamdhip64, and _C must bind
# to that same HIP runtime (same soname, already loaded) instead of pulling /opt/rocm's copy into
# the process as a second runtime — two runtimes in one process cannot share a device
# ("no ROCm-capable device is detected" from the second one).
import torch  # noqa: F401

_C = None
_ERR: Exception | None = None

try:  # pragma: no cover - exercised implicitly by every test
    _C = importlib.import_module("cuda_mpi_reductions_amd._C")
except ImportError as e:  # pragma: no cover
    _ERR = e


def native():
    """Return the loaded native module or raise a descriptive ImportError."""
    if _C is None:
        raise ImportError(
            "cuda_mpi_reductions_amd._C is not built (run `make python` or "
            "`python -c 'import __graft_entry__ as g; g.build()'`): %r" % (_ERR,)
        )
    return _C


def native_path() -> str:
    return os.path.abspath(native().__file__)


def available() -> bool:
    return _C is not None
