"""Single-GPU reductions with the native HIP kernels.

    python examples/01_single_gpu.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # in-tree package

import torch

from cuda_mpi_reductions_amd.ops import KernelConfig, Reducer, fill_, ladder_reduce, moments, reduce

dev = torch.device("cuda", 0)
x = fill_(torch.empty(1 << 28, dtype=torch.float64, device=dev), "uniform", seed=42)   # 2 GiB, U[0,1)

print("sum", reduce(x, "sum").item(), "min", reduce(x, "min").item(), "max", reduce(x, "max").item())
print("reference k6 (Harris ladder, 64 blocks):", ladder_reduce(x, "sum", kernel=6).item())
print("moments:", moments(x))

# explicit plan + timing
r = Reducer(dev, config=KernelConfig(block=512, unroll=16, wg_per_cu=1, nontemporal=True))
out = torch.empty(1, dtype=torch.float64, device=dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
r(x, "sum", out=out)
e0.record()
for _ in range(20):
    r(x, "sum", out=out)
e1.record()
e1.synchronize()
ms = e0.elapsed_time(e1) / 20
print(f"plan {r.last_plan}  {x.numel() * 8 / (ms * 1e-3) / 1e9:.1f} GB/s")
