"""Global sum of a sharded 1e9-element array: local HIP reduce + RCCL all-reduce over xGMI.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/02_distributed_sum.py
    (CPU only: torchrun --nproc-per-node 2 ... examples/02_distributed_sum.py --cpu)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # in-tree package

import sys
from dataclasses import replace

from cuda_mpi_reductions_amd.models import CONFIGS, ScalarReduction
from cuda_mpi_reductions_amd.parallel import dist as pdist

cpu = "--cpu" in sys.argv
ctx = pdist.init(device_type="cpu" if cpu else None)
cfg = CONFIGS["xgmi_1b_double_sum"]
if cpu:
    cfg = replace(cfg, n_total=1_000_000)
wl = ScalarReduction(cfg, ctx).setup()          # this rank's contiguous shard, filled on device
out = wl.new_slots(1)
work = wl.step(out)                             # local reduce + all-reduce of one element
if work is not None:
    work.wait()
check = wl.verify(out)
if ctx.is_root:
    print(f"{ctx.world_size} ranks: sum = {out.item():.6f}  verified={check['ok']}")
pdist.shutdown(ctx)
