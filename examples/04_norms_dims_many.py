"""MI355X additions beyond the reference: 16-bit inputs, fused norms, per-axis reductions and
one-launch reductions over a list of tensors.

    python examples/04_norms_dims_many.py
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/04_norms_dims_many.py   # sharded norms
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # in-tree package

import torch

from cuda_mpi_reductions_amd.ops import ReduceMany, norm, norm_many, reduce, reduce_dim, synthetic
from cuda_mpi_reductions_amd.parallel import dist as pdist

ctx = pdist.init()  # one rank (or torchrun's N ranks, RCCL over xGMI)
dev = ctx.device

# bf16 data, fp32 accumulation (every 16-bit value is exact in fp32)
w = synthetic(1 << 26, torch.bfloat16, device=dev, seed=ctx.rank) * 2 - 1
print(f"[rank {ctx.rank}] bf16 sum {reduce(w, 'sum').item():.4f}  amax {reduce(w, 'amax').item():.4f}")

# fused norms: one pass, no x*x temporary; with several ranks, of the whole sharded tensor
print(f"[rank {ctx.rank}] global L2 {norm(w).item():.4f}  global max|x| {norm(w, math.inf).item():.4f}")

# per-row / per-column reductions
m = w.view(1 << 13, 1 << 13)
row_max = reduce_dim(m, "max", dim=1)
col_sum = reduce_dim(m, "sum", dim=0)
print(f"[rank {ctx.rank}] rows {tuple(row_max.shape)} cols {tuple(col_sum.shape)}")

# a parameter-like list: bind once, relaunch each step (one kernel for the whole list)
params = [synthetic(n, torch.bfloat16, device=dev, seed=i) for i, n in enumerate([4096 * 4096, 4096, 11008 * 4096, 7])]
per_tensor = ReduceMany(params, "sumsq")
print(f"[rank {ctx.rank}] per-tensor sum of squares {per_tensor().tolist()}")
total, per = norm_many(params)
print(f"[rank {ctx.rank}] total grad-norm-style L2 over the list (all ranks) {total.item():.3f}")
torch.cuda.synchronize()
pdist.shutdown(ctx)
