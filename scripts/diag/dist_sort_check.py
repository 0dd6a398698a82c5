"""Diagnostic: the bench's --dist sort path (gloo control plane + nut_dist_create_rank) at
bench-like sizes: is the received range sorted and equal to the single-context sort?"""
import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
from nutdb_amd import Executor  # noqa: E402
from nutdb_amd.dist import NutDist  # noqa: E402
from nutdb_amd.workloads import SORT_COL, gen  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000_000
torch.cuda.set_device(0)
ex = Executor(0)
dist.init_process_group("gloo")
nd = NutDist.create_rank(1, 0, NutDist.unique_id(), 0)
col = gen(ex, SORT_COL, n)
ref = ex.sort_i64(col)
print("single:", ex.sort_stats())
for step in range(3):
    out = nd.sort_i64([col])[0]
    print("dist step", step, nd.sort_stats(), "equal:", bool(torch.equal(out, ref)),
          "distinct(first 1e6):", int(torch.unique(out[:1_000_000]).numel()))
nd.close()
ex.close()
dist.destroy_process_group()
