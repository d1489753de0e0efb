"""Arg-reductions: where the extreme is, not only what it is.

    python examples/05_argmax_maxloc.py
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/05_argmax_maxloc.py   # MPI_MAXLOC over GPUs
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/05_argmax_maxloc.py --cpu

* ``arg_reduce(x, "max", group=...)``: first index of the maximum of a whole array (+ its value);
  with ``group`` the array is every rank's shard concatenated in rank order (without it, rank-local);
* ``argmax(logits, dim=-1)``: per row — greedy decoding over a vocabulary, top-1 expert routing;
* ``loc_allreduce``: MPI_MAXLOC / MPI_MINLOC of per-rank (value, global index) pairs over RCCL.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # in-tree package

import torch

from cuda_mpi_reductions_amd.ops import arg_reduce, argmax, synthetic
from cuda_mpi_reductions_amd.parallel import dist as pdist

cpu = "--cpu" in sys.argv
ctx = pdist.init(device_type="cpu" if cpu else None)
dev = ctx.device
n = 1_000_000 if dev.type == "cpu" else 100_000_000

# this rank's shard; its local extreme is a one-row arg-reduction (dim=-1 never goes global)
x = synthetic(n, torch.float64, device=dev, seed=ctx.rank)
lv, li = arg_reduce(x.view(1, -1), "max", dim=-1)
print(f"[rank {ctx.rank}] local max {lv.item():.12f} at {li.item()} (torch: {int(x.argmax())})")

# per row: 64 tokens of 128k-vocabulary bf16 logits, 4096 tokens routed over 64 experts
vocab = 8192 if dev.type == "cpu" else 131_072
logits = synthetic(64 * vocab, torch.bfloat16, device=dev, seed=7).view(64, vocab)
tokens = argmax(logits, dim=-1)
router = synthetic(4096 * 64, torch.bfloat16, device=dev, seed=8).view(4096, 64)
experts = argmax(router, dim=-1)
match = bool(torch.equal(tokens, logits.argmax(-1)) and torch.equal(experts, router.argmax(-1)))
print(f"[rank {ctx.rank}] greedy tokens {tokens[:4].tolist()}  experts {experts[:8].tolist()} (match torch: {match})")

# MPI_MAXLOC across ranks: every rank learns the global max and its global index (shards in rank order)
offset = ctx.rank * n
gv, gi = pdist.loc_allreduce(lv, li + offset, "max") if ctx.world_size > 1 else (lv, li + offset)
# the same answer in one call: a whole-array arg_reduce over the group's shards
av, ai = arg_reduce(x, "max", group=torch.distributed.group.WORLD)
ok = gv.item() == av.item() and gi.item() == ai.item()
print(f"[rank {ctx.rank}] global max {gv.item():.12f} at global index {gi.item()} "
      f"of {ctx.world_size} shards (arg_reduce agrees: {ok})")
if dev.type == "cuda":
    torch.cuda.synchronize()
pdist.shutdown(ctx)
