"""Tensor-level reductions backed by the native gfx950 kernels.

Reference parity: ``{sum,min,max}reduce<T>`` launch templates (cuda/C/src/reduction/reduction.h:15-25)
and the CPU references ``sumreduceCPU``/``minreduceCPU``/``maxreduceCPU``
(cuda/C/src/reduction/reduction.cpp:214-249).

* device tensors  -> ``_C.reduce`` (one-launch single-pass kernel, csrc/kernels/reduce.hip)
* host tensors    -> ``_C.cpu_reduce`` (compensated / exact native reference, multi-threaded)
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Optional

import torch

from .._native import native

__all__ = [
    "DTYPE_CODES",
    "OP_CODES",
    "KernelConfig",
    "Reducer",
    "reduce",
    "reduce_partials",
    "default_acc_dtype",
    "dtype_code",
    "op_code",
    "cpu_reduce",
    "sum_tolerance",
    "ladder_reduce",
    "FaninError",
]


class FaninError(RuntimeError):
    """A device reduction's fan-in reached its wait bound: the result is poisoned (NaN for floating
    accumulators, the operator's identity for integers — which no value check can tell apart from
    a real result, so the workspace's error word is the signal)."""

DTYPE_CODES = {torch.int32: 0, torch.int64: 1, torch.float32: 2, torch.float64: 3,
               torch.bfloat16: 4, torch.float16: 5}
CODE_DTYPES = {v: k for k, v in DTYPE_CODES.items()}
# sum / min / max are the reference's operators; sumsq (fused sum of squares) and amax (fused
# max |x|) transform each element once as it is loaded (floating dtypes only).
OP_CODES = {"sum": 0, "min": 1, "max": 2, "sumsq": 3, "amax": 4}
XCD_SKEW_AUTO = -(2 ** 31)  # ReduceConfig::xcd_skew's "tuned default"
FUSED_OPS = ("sumsq", "amax")


def fan_error_message(word: int) -> str:
    """What a non-zero Workspace::error() word means (csrc/include/mireduce/reduce.hpp)."""
    msgs = []
    if word & 1:
        msgs.append("polled fan-in: a launch reached its wait bound")
    if word & 2:
        msgs.append("XCD-weighted split: a workgroup waited past the bound for the XCD anchor (its tiles were "
                    "not the split's)")
    if word & ~3:
        msgs.append(f"fan-in error word {word:#x}")
    return "; ".join(msgs) + " (results poisoned since; workspace reset)"


def dtype_code(dt: torch.dtype) -> int:
    try:
        return DTYPE_CODES[dt]
    except KeyError:
        raise TypeError(f"unsupported dtype {dt}; supported: int32, int64, float32, float64, "
                        "bfloat16, float16") from None


def op_code(op: str) -> int:
    try:
        return OP_CODES[op.lower()]
    except KeyError:
        raise ValueError(f"unsupported op {op!r}; supported: {', '.join(OP_CODES)}") from None


def default_acc_dtype(dt: torch.dtype, op: str) -> torch.dtype:
    """int32 SUM -> int64, float32 SUM / SUMSQ -> float64, bfloat16/float16 -> float32 (every op),
    everything else keeps its dtype."""
    if op.lower() in FUSED_OPS and not dt.is_floating_point:
        raise TypeError(f"{op} needs a floating-point tensor, got {dt}")
    return CODE_DTYPES[native().default_acc(dtype_code(dt), op_code(op))]


@dataclass
class KernelConfig:
    """Tunables of the streaming kernel (0 = tuned default; see docs/TUNING.md)."""

    block: int = 0
    unroll: int = 0
    wg_per_cu: int = 0
    max_blocks: int = 0
    nontemporal: Optional[bool] = None  # None: size-dependent tuned choice
    single_pass: bool = True
    window: Optional[int] = None        # loads in flight per thread: None tuned, 0 hipcc's schedule, 2 | 4
    xcd_skew: Optional[int] = None      # XCD-weighted split, permille of rounds (+: odd XCCs more); None tuned
    segment_bytes: int = 0              # segmented launches: 0 auto (8 GiB above 16 GiB), < 0 one launch, > 0 size

    @property
    def policy(self) -> int:
        return -1 if self.nontemporal is None else int(bool(self.nontemporal))

    def kwargs(self) -> dict:
        return dict(
            block=self.block,
            unroll=self.unroll,
            wg_per_cu=self.wg_per_cu,
            max_blocks=self.max_blocks,
            policy=self.policy,
            single_pass=self.single_pass,
            window=-1 if self.window is None else int(self.window),
            xcd_skew=XCD_SKEW_AUTO if self.xcd_skew is None else int(self.xcd_skew),
            segment_bytes=int(self.segment_bytes),
        )


def _stream_handle(device: torch.device, stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return int(s.cuda_stream)


class Reducer:
    """A per-device reduction engine owning its scratch workspace.

    One ``Reducer`` must not run two reductions concurrently on different streams (the
    workspace's arrival tickets are shared); create one per stream for concurrent use.
    """

    def __init__(self, device=None, max_grid: int = 16384, config: Optional[KernelConfig] = None):
        C = native()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("Reducer needs a GPU device")
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        self.ws = C.Workspace(idx, max_grid)
        self.config = config or KernelConfig()
        self.last_plan: dict = {}

    @property
    def num_cus(self) -> int:
        return self.ws.num_cus

    def check(self, stream: Optional[torch.cuda.Stream] = None) -> Optional[str]:
        """None, or the polled fan-in's sticky error: some launch's finisher reached its wait bound
        (a workgroup never published), so that launch and every later one on this workspace wrote a
        poisoned result — NaN for floating accumulators, the operator's identity for integers, for
        which only this error word tells the result is bad. Synchronises the device; after an error
        the workspace is reset, so the next launch is good."""
        torch.cuda.synchronize(self.device)
        word = self.ws.error()
        if word == 0:
            return None
        self.ws.reset(_stream_handle(self.device, stream))
        torch.cuda.synchronize(self.device)
        return fan_error_message(word)

    def __call__(
        self,
        x: torch.Tensor,
        op: str = "sum",
        acc_dtype: Optional[torch.dtype] = None,
        out: Optional[torch.Tensor] = None,
        stream: Optional[torch.cuda.Stream] = None,
        config: Optional[KernelConfig] = None,
        check: bool = False,
    ) -> torch.Tensor:
        """Enqueue the reduction (asynchronous). ``check=True`` makes the call synchronous and raises
        :class:`FaninError` when the workspace's sticky error is set (the result is poisoned; the
        workspace is reset first, so the next call is good). Without it, call :meth:`check`
        before trusting an integer result."""
        C = native()
        if x.device != self.device:
            raise ValueError(f"tensor on {x.device}, reducer on {self.device}")
        if not x.is_contiguous():
            x = x.contiguous()
        acc = acc_dtype or default_acc_dtype(x.dtype, op)
        if out is None:
            out = torch.empty(1, dtype=acc, device=self.device)
        elif out.dtype != acc or out.device != self.device or out.numel() < 1:
            raise ValueError("out must be a 1+ element tensor of the accumulator dtype on the same device")
        cfg = config or self.config
        self.last_plan = C.reduce(
            self.ws,
            x.data_ptr(),
            x.numel(),
            dtype_code(x.dtype),
            op_code(op),
            dtype_code(acc),
            out.data_ptr(),
            _stream_handle(self.device, stream),
            **cfg.kwargs(),
        )
        if check:
            err = self.check(stream)
            if err is not None:
                raise FaninError(err)
        return out

    def bind(self, x: torch.Tensor, op: str = "sum", acc_dtype: Optional[torch.dtype] = None,
             out: Optional[torch.Tensor] = None, config: Optional[KernelConfig] = None, xrank=None):
        """Resolve plan, kernel variant and arguments once (``_C.BoundReduce``).

        ``bound.launch(stream_handle[, out_ptr])`` is then a single kernel launch with no planning
        or argument marshalling — the per-step path of bench loops and hipGraph capture. ``x``,
        ``out`` and this Reducer must outlive the returned object.

        ``xrank`` (a connected ``_C.XrankChannel``, see :mod:`parallel.xrank`): every launch then
        also folds all ranks' partials in-kernel, so ``out`` receives the GLOBAL result — every rank
        must launch its bound reductions of that channel in the same order.
        """
        C = native()
        if x.device != self.device or not x.is_contiguous():
            raise ValueError("bind needs a contiguous tensor on the reducer's device")
        acc = acc_dtype or default_acc_dtype(x.dtype, op)
        if out is None:
            out = torch.empty(1, dtype=acc, device=self.device)
        elif out.dtype != acc or out.device != self.device or out.numel() < 1:
            raise ValueError("out must be a 1+ element tensor of the accumulator dtype on the same device")
        cfg = config or self.config
        if xrank is not None and not xrank.connected:
            raise ValueError("bind: the XrankChannel is not connected")
        b = C.BoundReduce(self.ws, x.data_ptr(), x.numel(), dtype_code(x.dtype), op_code(op), dtype_code(acc),
                          out.data_ptr(), xrank=xrank.desc_ptr if xrank is not None else 0, **cfg.kwargs())
        self.last_plan = b.plan
        return b


_reducers: dict = {}
_lock = threading.Lock()


def _default_reducer(device: torch.device) -> Reducer:
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    with _lock:
        r = _reducers.get(key)
        if r is None:
            if torch.cuda.is_current_stream_capturing():
                # A new Reducer allocates and zeroes its workspace synchronously, which would
                # invalidate the capture: make it before capturing.
                raise RuntimeError("reduce(): first call on this stream inside a hipGraph capture; call reduce() "
                                   "once on the capture stream before capturing, or capture a Reducer / "
                                   "Reducer.bind() launch created beforehand")
            r = Reducer(device)
            _reducers[key] = r
        return r


def cpu_reduce(x: torch.Tensor, op: str = "sum", acc_dtype: Optional[torch.dtype] = None, threads: int = 0):
    """Native host reference: returns a Python int/float (exact ints, compensated floats)."""
    C = native()
    if x.device.type != "cpu":
        raise ValueError("cpu_reduce needs a host tensor")
    x = x.contiguous()
    acc = acc_dtype or default_acc_dtype(x.dtype, op)
    return C.cpu_reduce(x.data_ptr(), x.numel(), dtype_code(x.dtype), op_code(op), dtype_code(acc), threads)


def reduce(
    x: torch.Tensor,
    op: str = "sum",
    acc_dtype: Optional[torch.dtype] = None,
    out: Optional[torch.Tensor] = None,
    config: Optional[KernelConfig] = None,
    check: bool = False,
) -> torch.Tensor:
    """Reduce all elements of ``x`` with ``op`` into a 1-element tensor of the accumulator dtype.

    Device tensors run the native HIP kernel on the current stream (asynchronous). Host tensors
    run the native CPU reference. ``check=True`` (device tensors): wait for the result and raise
    :class:`FaninError` if the kernel's fan-in failed — the only way to tell for integer results,
    whose poisoned value is the operator's identity.
    """
    if x.device.type == "cuda":
        return _default_reducer(x.device)(x, op, acc_dtype, out, config=config, check=check)
    acc = acc_dtype or default_acc_dtype(x.dtype, op)
    val = cpu_reduce(x, op, acc)
    res = torch.tensor([val], dtype=acc)
    if out is not None:
        out.copy_(res)
        return out
    return res


def reduce_partials(x: torch.Tensor, op: str = "sum", acc_dtype=None, max_grid: int = 16384,
                    config: Optional[KernelConfig] = None):
    """First level only (the reference's --cpufinal path): returns the per-workgroup partials."""
    C = native()
    if x.device.type != "cuda":
        raise ValueError("reduce_partials needs a device tensor")
    acc = acc_dtype or default_acc_dtype(x.dtype, op)
    cfg = config or KernelConfig()
    parts = torch.empty(max_grid, dtype=acc, device=x.device)
    info = torch.cuda.get_device_properties(x.device)
    plan = C.reduce_partials(
        x.data_ptr(), x.numel(), dtype_code(x.dtype), op_code(op), dtype_code(acc), parts.data_ptr(),
        max_grid, info.multi_processor_count, _stream_handle(x.device, None),
        block=cfg.block, unroll=cfg.unroll, wg_per_cu=cfg.wg_per_cu, max_blocks=cfg.max_blocks,
        policy=cfg.policy,
    )
    return parts[: plan["grid"]], plan


def sum_tolerance(dtype: torch.dtype, acc: torch.dtype, n: int, abs_sum: float) -> float:
    return native().sum_tolerance(dtype_code(dtype), dtype_code(acc), n, abs_sum)


def ladder_reduce(x: torch.Tensor, op: str = "sum", kernel: int = 6, acc_dtype=None, threads: int = 256,
                  max_blocks: int = 64) -> torch.Tensor:
    """Reduce with one of the Harris-ladder kernels 0..6 (csrc/kernels/ladder.hip), multi-pass like
    the reference's benchmarkReduce* relaunch loop (reduction.cpp:344-357)."""
    C = native()
    if x.device.type != "cuda":
        raise ValueError("ladder_reduce needs a device tensor")
    x = x.contiguous()
    acc = acc_dtype or default_acc_dtype(x.dtype, op)
    out = torch.empty(1, dtype=acc, device=x.device)
    nbytes = C.ladder_scratch_bytes(kernel, x.numel(), threads, max_blocks)
    scratch = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=x.device)
    C.ladder_reduce(kernel, x.data_ptr(), x.numel(), dtype_code(x.dtype), op_code(op), dtype_code(acc),
                    out.data_ptr(), scratch.data_ptr(), threads, max_blocks, _stream_handle(x.device, None))
    return out
