#!/usr/bin/env python3
"""How long does a torch pass over the array slow the streaming kernel that follows it?

profiles/r3_selfcheck/: a torch reference pass (bf16 -> fp64 chunks) right before the timed steps
cost the bf16 bench 6 % for the whole timed run. This probe times the same bound reduction
(hipEvent per launch) after each of these preludes:

    A  nothing (baseline)              D  torch pass, then 100 untimed launches
    B  torch pass                      E  torch pass, then torch.cuda.empty_cache()
    C  torch pass, then 0.5 s idle     F  torch's own bf16 sum (no fp64 temporaries)
    G  E, then 0.5 s idle              H  torch pass in 16M-element chunks, then empty_cache()

    python tools/settle_probe.py [--n 4e9] [--dtype bfloat16] [--steps 30] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cuda_mpi_reductions_amd.ops import Reducer, default_acc_dtype, fill_  # noqa: E402

DT = {"bfloat16": torch.bfloat16, "float32": torch.float32, "float64": torch.float64}


def torch_pass(x: torch.Tensor, chunk: int = 1 << 28) -> float:
    """The bench's reference (models/workloads.py ScalarReduction.reference): fp64 sum and |x| sum."""
    s = torch.zeros(1, dtype=torch.float64, device=x.device)
    for i in range(0, x.numel(), chunk):
        c = x[i:i + chunk]
        s += c.sum(dtype=torch.float64)
        s += c.abs().sum(dtype=torch.float64)
    return s.item()


def clocks() -> str:
    try:
        r = subprocess.run(["rocm-smi", "--showclocks"], capture_output=True, text=True, timeout=20)
        return " | ".join(ln.strip() for ln in r.stdout.splitlines() if "sclk" in ln or "mclk" in ln)[:300]
    except Exception as e:  # noqa: BLE001 - diagnostics only
        return f"(rocm-smi unavailable: {e})"


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=float, default=4e9)
    p.add_argument("--dtype", default="bfloat16", choices=sorted(DT))
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--json", default="")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    dt = DT[a.dtype]
    x = torch.empty(int(a.n), dtype=dt, device=dev)
    fill_(x, "uniform", seed=5)
    acc = default_acc_dtype(dt, "sum")
    out = torch.empty(1, dtype=acc, device=dev)
    red = Reducer(dev)  # must outlive the bound launch
    bound = red.bind(x, "sum", acc, out=out)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    sh = torch.cuda.current_stream(dev).cuda_stream

    def timed(extra: int = 0) -> list:
        for _ in range(extra):
            bound.launch(sh)
        ev[0].record()
        for i in range(a.steps):
            bound.launch(sh)
            ev[i + 1].record()
        ev[-1].synchronize()
        return [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(a.steps)]

    nbytes = x.numel() * x.element_size()
    timed()  # warm-up
    torch.cuda.synchronize()
    res = {}
    for name in "ABCDEFGH":
        if name != "A":
            if name == "F":
                x.sum().item()
            else:
                torch_pass(x, chunk=1 << 24 if name == "H" else 1 << 28)
        if name in ("E", "G", "H"):
            torch.cuda.empty_cache()
        if name in ("C", "G"):
            time.sleep(0.5)
        us = timed(100 if name == "D" else 0)
        med = statistics.median(us)
        res[name] = {"median_us": round(med, 1), "TBps": round(nbytes / med / 1e6, 3),
                     "first5_us": [round(v, 1) for v in us[:5]], "last5_us": [round(v, 1) for v in us[-5:]],
                     "clocks_after": clocks()}
        print(f"{name}: median {med:9.1f} us = {nbytes / med / 1e6:6.3f} TB/s   first {res[name]['first5_us']}  "
              f"last {res[name]['last5_us']}", flush=True)
        print(f"   {res[name]['clocks_after']}", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"n": int(a.n), "dtype": a.dtype, "steps": a.steps, "phases": res}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
