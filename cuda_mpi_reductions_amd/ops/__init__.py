"""Tensor operations backed by the native gfx950 kernels (csrc/kernels)."""
from .reduce import (  # noqa: F401
    DTYPE_CODES, OP_CODES, FaninError, KernelConfig, Reducer, cpu_reduce, default_acc_dtype, dtype_code,
    ladder_reduce, op_code, reduce, reduce_partials, sum_tolerance,
)
from .fill import PATTERNS, fill_, mt19937_fill_, synthetic  # noqa: F401
from .moments import combine_moments, moments  # noqa: F401
from .reduce_dim import reduce_dim  # noqa: F401
from .norm import norm  # noqa: F401
from .reduce_many import ReduceMany, norm_many, reduce_many  # noqa: F401
from .arg_reduce import arg_reduce, argmax, argmin  # noqa: F401
