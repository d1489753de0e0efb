"""Cross-GPU reductions over xGMI without RCCL: the fused in-kernel finish and the direct collective.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/06_xgmi_collectives.py
    python examples/06_xgmi_collectives.py                          # one GPU (world of 1)
    MIREDUCE_FORCE_DEVICE=0 torchrun --nproc-per-node 4 ... 06_xgmi_collectives.py --backend gloo
                                                                   # 4 ranks sharing one GPU

1. Global sum of a sharded array in ONE kernel per reduction: the reduction's last workgroup
   pushes its partial into every rank's IPC-mapped mailbox and folds all ranks' partials
   (``Reducer.bind(..., xrank=open_channel(dev))``) — bit-identical on every rank, graph-capturable.
2. reduce.c's element-wise reduce (mpi/reduce.c:76,90) with the one-kernel direct collective
   (``DirectComm``): every rank pulls its chunk from all peers at once, device-side barriers.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # in-tree package

import torch

from cuda_mpi_reductions_amd.ops import Reducer, fill_
from cuda_mpi_reductions_amd.parallel import DirectComm, check_channel, open_channel
from cuda_mpi_reductions_amd.parallel import dist as pdist

backend = sys.argv[sys.argv.index("--backend") + 1] if "--backend" in sys.argv else None
ctx = pdist.init(backend=backend)
dev = ctx.device

# ---- 1. one kernel per global reduction -------------------------------------------------------
n_total = 200_000_000
offset, count = pdist.shard(n_total, ctx.rank, ctx.world_size)
x = fill_(torch.empty(count, dtype=torch.float64, device=dev), "uniform", seed=11, offset=offset)
ch = open_channel(dev)                                  # collective: mailboxes mapped on every rank
out = torch.empty(1, dtype=torch.float64, device=dev)
bound = Reducer(dev).bind(x, "sum", out=out, xrank=ch)  # every launch writes the GLOBAL sum
stream = torch.cuda.current_stream(dev).cuda_stream
for _ in range(10):
    bound.launch(stream)
torch.cuda.synchronize(dev)
ref = torch.tensor([x.sum().item()], dtype=torch.float64, device="cpu" if ctx.backend == "gloo" else dev)
if ctx.world_size > 1:
    torch.distributed.all_reduce(ref)
err = check_channel([ch])
print(f"[rank {ctx.rank}] fused global sum {out.item():.6f} (torch: {ref.item():.6f}, "
      f"epoch {ch.epoch()}, channel {'ok' if err is None else err})")

# ---- 2. reduce.c's element-wise reduce to rank 0 with the direct collective -------------------
per_rank = 1 << 22
v = fill_(torch.empty(per_rank, dtype=torch.float64, device=dev), "uniform", seed=100 + ctx.rank)
comm = DirectComm(dev, v.numel() * v.element_size())   # collective: buffers mapped on every rank
res = v.clone()
comm.reduce(res, "sum", root=0)                        # one kernel: reduce-scatter + gather to root
torch.cuda.synchronize(dev)
parts = [torch.empty_like(v) for _ in range(ctx.world_size)]
if ctx.world_size > 1 and ctx.backend == "nccl":
    torch.distributed.all_gather(parts, v)
elif ctx.world_size > 1:
    cpu_parts = [torch.empty(per_rank, dtype=torch.float64) for _ in range(ctx.world_size)]
    torch.distributed.all_gather(cpu_parts, v.cpu())
    parts = [p.to(dev) for p in cpu_parts]
else:
    parts = [v]
if ctx.rank == 0:
    exp = torch.stack(parts).sum(0)
    ok = bool(torch.allclose(res, exp, rtol=1e-12, atol=1e-12))
    print(f"[rank 0] direct element-wise reduce of {ctx.world_size} x {per_rank} doubles: "
          f"{'matches' if ok else 'DIFFERS FROM'} the gathered sum; {comm.check() or 'no timeouts'}")
else:
    comm.check()  # (collective)
pdist.shutdown(ctx)
