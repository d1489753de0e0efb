#!/usr/bin/env python3
"""Host issue cost of one bench step, and what hipGraph replay buys.

At N GPUs each rank's bench step is a 1e9/N-double local reduce (0.14 ms at N=8) plus a
1-element RCCL all-reduce. If issuing a step from Python costs more host time than the GPU
spends on it, the GPU starves and strong scaling stalls. This measures, per variant and array
size, the host time to enqueue K steps (GPU kept busy) and the GPU time per step:

  eager          Reducer call only (N=1 bench step)
  eager+ar       Reducer + async dist.all_reduce of the slot (N>1 bench step; here world 1)
  bound          the prepared native launch (_C.BoundReduce) instead of the generic call
  bound+ar       prepared launch + all_reduce
  graph          torch.cuda.CUDAGraph of CHUNK eager steps, replayed K/CHUNK times
  graph+ar       same with the all-reduce captured too
  graph2         two lanes (own workspaces) alternating on two forked streams inside the graph

Usage (GPU box): python tools/host_overhead.py [--sizes 1048576,125000000] [--steps 400]
Prints one JSON line per (variant, size).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cuda_mpi_reductions_amd._native import native  # noqa: E402
from cuda_mpi_reductions_amd.ops import Reducer, fill_  # noqa: E402
from cuda_mpi_reductions_amd.parallel import dist as pdist  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1048576,125000000")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--chunk", type=int, default=8)
    ap.add_argument("--variants", default="eager,eager+ar,bound,bound+ar,graph,graph+ar,graph2")
    a = ap.parse_args()
    ctx = pdist.init()
    dev = ctx.device
    C = native()
    K = a.steps - a.steps % a.chunk
    for n in [int(s) for s in a.sizes.split(",")]:
        x = torch.empty(n, dtype=torch.float64, device=dev)
        fill_(x, "uniform", seed=7)
        r = Reducer(dev)
        slots = torch.zeros(a.chunk, dtype=torch.float64, device=dev)
        bound = [C.BoundReduce(r.ws, x.data_ptr(), n, 3, 0, 3, slots[i:i + 1].data_ptr())
                 for i in range(a.chunk)] if hasattr(C, "BoundReduce") else None
        r2 = Reducer(dev)  # second workspace for the two-lane graph
        lane2 = C.BoundReduce(r2.ws, x.data_ptr(), n, 3, 0, 3, slots[0:1].data_ptr())
        ref = x.sum().item()

        def eager(i, ar):
            r(x, "sum", torch.float64, out=slots[i % a.chunk:i % a.chunk + 1])
            return pdist.scalar_allreduce(slots[i % a.chunk:i % a.chunk + 1], "sum", async_op=True) if ar else None

        def bnd(i, ar):
            bound[i % a.chunk].launch(torch.cuda.current_stream(dev).cuda_stream)
            return pdist.scalar_allreduce(slots[i % a.chunk:i % a.chunk + 1], "sum", async_op=True) if ar else None

        def graph2_capture():
            # two lanes (own workspace each) on two forked streams, alternating steps: kernel j+1
            # may start while kernel j drains / finalises
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream(dev)
            with torch.cuda.graph(g):
                main = torch.cuda.current_stream(dev)
                side.wait_stream(main)
                for i in range(a.chunk):
                    if i % 2 == 0:
                        bound[0].launch(main.cuda_stream, slots[i:i + 1].data_ptr())
                    else:
                        lane2.launch(side.cuda_stream, slots[i:i + 1].data_ptr())
                main.wait_stream(side)
            return g

        for v in a.variants.split(","):
            ar = v.endswith("+ar")
            base = v.split("+")[0]
            if base == "bound" and bound is None:
                continue
            try:
                if base == "graph2":
                    g = graph2_capture()
                    fn = lambda: [g.replay() for _ in range(K // a.chunk)]  # noqa: E731
                elif base == "graph":
                    g = torch.cuda.CUDAGraph()
                    s = torch.cuda.Stream(dev)
                    s.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.stream(s):
                        for i in range(a.chunk):  # warm-up outside capture on the side stream
                            w = eager(i, ar)
                            if w is not None:
                                w.wait()
                    torch.cuda.current_stream(dev).wait_stream(s)
                    torch.cuda.synchronize(dev)
                    with torch.cuda.graph(g):
                        works = [eager(i, ar) for i in range(a.chunk)]
                        for w in works:
                            if w is not None:
                                w.wait()
                    fn = lambda: [g.replay() for _ in range(K // a.chunk)]  # noqa: E731
                else:
                    step = eager if base == "eager" else bnd

                    def fn():
                        works = [step(i, ar) for i in range(K)]
                        for w in works:
                            if w is not None:
                                w.wait()
                fn()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                fn()
                t1 = time.perf_counter()
                torch.cuda.synchronize(dev)
                t2 = time.perf_counter()
                ok = bool((slots - ref).abs().max().item() <= 1e-9 * abs(ref) + 1e-6)
                rec = {"variant": v, "n": n, "steps": K, "issue_us_per_step": round((t1 - t0) / K * 1e6, 2),
                       "ms_per_step": round((t2 - t0) / K * 1e3, 5),
                       "gbps": round(n * 8 * K / (t2 - t0) / 1e9, 1), "ok": ok}
            except Exception as e:  # report and continue with the next variant
                torch.cuda.synchronize(dev)
                rec = {"variant": v, "n": n, "error": f"{type(e).__name__}: {e}"[:300]}
            print(json.dumps(rec), flush=True)
    pdist.shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
