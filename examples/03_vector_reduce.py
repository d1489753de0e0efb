"""reduce.c semantics: each rank holds N/P elements; element-wise reduce to rank 0.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/03_vector_reduce.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # in-tree package

from dataclasses import replace

from cuda_mpi_reductions_amd.models import CONFIGS, VectorReduction
from cuda_mpi_reductions_amd.parallel import dist as pdist

ctx = pdist.init(device_type="cpu")
for op in ("max", "min", "sum"):                 # reduce.c's order (mpi/reduce.c:26-28)
    cfg = replace(CONFIGS["mpi_1m_int32_sum_cpu2"], op=op)
    wl = VectorReduction(cfg, ctx).setup(mt19937=True)   # reduce.c's per-rank MT19937 data
    wl.step()
    ok = wl.verify()["ok"]
    if ctx.is_root:
        print(f"INT {op.upper()} {ctx.world_size}: first elements {wl.y[:3].tolist()} verified={ok}")
pdist.shutdown(ctx)
