"""Python front-end with the reference's command-line grammar and output lines.

    python -m cuda_mpi_reductions_amd --method=SUM --type=double --n=268435456 [--iterations=100]
        [--qatest] [--device=0] [--acc=double] [--pattern=smallint|uniform|fullrange|iotamod] [--json=PATH]
        [--arg]   (with MIN/MAX: the first index of the extreme too — ops.arg_reduce)

Same flags and lines as the native `reduction` app (cuda/C/src/reduction/reduction.cpp:84-204):
QA banner, "METHOD: ...", "<n> elements", the "Reduction, Throughput = ..." line (GB = 1e9 B),
"GPU result = / CPU result =", and the QA status. Runs the native HIP kernel through
cuda_mpi_reductions_amd.ops; verification uses torch's own fp64/int64 reduction.
"""
from __future__ import annotations

import json
import sys

from .utils import cli
from .utils.formats import throughput_line

_TYPES = {"int": "int32", "int32": "int32", "int64": "int64", "long": "int64", "float": "float32",
          "float32": "float32", "double": "float64", "float64": "float64", "bf16": "bfloat16",
          "bfloat16": "bfloat16", "half": "float16", "fp16": "float16", "float16": "float16"}


def _qa(argv, status=None):
    exe = "cuda_mpi_reductions_amd"
    qatest = any(a.lstrip("-").split("=")[0].lower() == "qatest" for a in argv)
    if status is None:
        print(("&&&& RUNNING " + " ".join([exe] + argv)) if qatest else f"[{exe}] starting...", file=sys.stderr)
    else:
        print((f"&&&& {status} " + " ".join([exe] + argv)) if qatest else f"[{exe}] test results...\n{status}",
              file=sys.stderr)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    _qa(argv)
    try:
        args = cli.parse(argv)
    except cli.CliError as e:
        print(str(e), file=sys.stderr)
        return 1
    if cli.has(args, "help"):
        print(__doc__)
        return 0
    method = cli.get_str(args, "method")
    if not cli.has(args, "method"):
        print("MISSING --method FLAG.\nYou must provide --method={ SUM | MIN | MAX }.", file=sys.stderr)
        return 1
    if method not in ("SUM", "MIN", "MAX", "SUMSQ", "AMAX"):
        print("No --method specified!", file=sys.stderr)
        return 1
    import torch

    from .ops import KernelConfig, Reducer, fill_
    from .ops.reduce import default_acc_dtype, sum_tolerance
    tname = (cli.get_str(args, "type") or "int").lower()
    dt = getattr(torch, _TYPES.get(tname, "int32"))
    op = method.lower()
    n = cli.get_int(args, "n", 1 << 24)
    iters = cli.get_int(args, "iterations", 100)
    dev_idx = cli.get_int(args, "device", 0)
    if not torch.cuda.is_available() or dev_idx >= torch.cuda.device_count():
        print("Error: no usable HIP device.", flush=True)
        _qa(argv, "WAIVED")
        return 0
    dev = torch.device("cuda", dev_idx)
    torch.cuda.set_device(dev)
    acc_name = cli.get_str(args, "acc")
    acc = getattr(torch, _TYPES[acc_name.lower()]) if acc_name else default_acc_dtype(dt, op)
    print(f"Using Device {dev_idx}: {torch.cuda.get_device_name(dev)}\n")
    print(f"Reducing array of type {tname}\n")
    print(f"METHOD: {method}\n{n} elements")
    x = torch.empty(n, dtype=dt, device=dev)
    fill_(x, cli.get_str(args, "pattern") or "smallint", seed=cli.get_int(args, "seed", 1))
    if cli.has(args, "arg"):
        return _arg_main(argv, args, x, op, iters)
    r = Reducer(dev, config=KernelConfig())
    out = torch.empty(1, dtype=acc, device=dev)
    r(x, op, acc, out=out)  # warm-up
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        r(x, op, acc, out=out)
    e1.record()
    e1.synchronize()
    secs = e0.elapsed_time(e1) / iters * 1e-3
    nbytes = n * x.element_size()
    plan = r.last_plan
    print(f"{plan.get('grid', 0)} blocks\n")
    print(throughput_line(1e-9 * nbytes / secs if secs else 0.0, secs, n, 1, plan.get("block", 0)))
    got = out.item()
    if op == "sumsq":
        xd = x.double()
        ref = (xd * xd).sum().item()
        ok = abs(got - ref) <= sum_tolerance(dt, acc, n, ref)
    elif op == "amax":
        ref = x.abs().max().item()
        ok = got == ref
    elif op == "sum":
        ref = x.sum(dtype=torch.float64 if acc.is_floating_point else torch.int64).item()
        if acc == torch.int32:
            ref = (int(ref) + 2 ** 31) % 2 ** 32 - 2 ** 31
        tol = sum_tolerance(dt, acc, n, x.abs().sum(dtype=torch.float64).item()) if acc.is_floating_point else 0
        ok = abs(got - ref) <= tol
    else:
        ref = (x.min() if op == "min" else x.max()).item()
        ok = got == ref
    print(f"\nGPU result = {got}\nCPU result = {ref}\n")
    jpath = cli.get_str(args, "json")
    if jpath:
        with open(jpath, "a") as f:
            f.write(json.dumps({"app": "python-reduction", "method": method, "type": tname, "n": n,
                                "gb_per_s": 1e-9 * nbytes / secs if secs else None, "avg_s": secs,
                                "plan": plan, "verified": bool(ok)}) + "\n")
    _qa(argv, "PASSED" if ok else "FAILED")
    return 0 if ok else 1


def _arg_main(argv, args, x, op, iters) -> int:
    """--arg: time ops.arg_reduce (first index of the MIN/MAX) and check it against torch.argmin/argmax."""
    import torch

    from .ops import arg_reduce
    if op not in ("min", "max"):
        print("error: --arg needs --method=MIN or MAX", file=sys.stderr)
        _qa(argv, "FAILED")
        return 1
    arg_reduce(x, op)  # warm-up
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        v, i = arg_reduce(x, op)
    e1.record()
    e1.synchronize()
    secs = e0.elapsed_time(e1) / iters * 1e-3
    n, nbytes = x.numel(), x.numel() * x.element_size()
    print(throughput_line(1e-9 * nbytes / secs if secs else 0.0, secs, n, 1, 256))
    ref = int((x.argmax() if op == "max" else x.argmin()).item())
    got = int(i.item())
    ok = got == ref
    print(f"\nGPU result = index {got}\nCPU result = index {ref}\n")
    jpath = cli.get_str(args, "json")
    if jpath:
        with open(jpath, "a") as f:
            f.write(json.dumps({"app": "python-reduction", "method": "ARG" + op.upper(), "n": n,
                                "gb_per_s": 1e-9 * nbytes / secs if secs else None, "avg_s": secs, "index": got,
                                "verified": bool(ok)}) + "\n")
    _qa(argv, "PASSED" if ok else "FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
