"""Diagnostic: host-side time split of a large-G group-by step (nut_groupby, result to host, free)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np
import torch

from nutdb_amd import Agg, AggQuery, Executor
from nutdb_amd.workloads import gen, groupby_cols

G = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
n = 1_000_000_000
ex = Executor(0)
key, val = [gen(ex, s, n) for s in groupby_cols(G, dyadic=True)]
torch.cuda.synchronize()
q = AggQuery(keys=[key], values=[val], aggs=[Agg("sum", "col", (0,))])
for it in range(4):
    t0 = time.perf_counter()
    g = ex.groupby(q, group_hint=G)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    m = len(g)
    t2 = time.perf_counter()
    k = np.zeros((m, 1), dtype=np.int64)
    a = np.zeros((m, 1), dtype=np.uint64)
    t3 = time.perf_counter()
    from nutdb_amd._lib import lib
    lib.nut_groups_to_host(g.h, k.ctypes.data, a.ctypes.data, m)
    t4 = time.perf_counter()
    g.free()
    t5 = time.perf_counter()
    print(f"groupby {1e3*(t1-t0):.2f} size {1e3*(t2-t1):.2f} alloc {1e3*(t3-t2):.2f} to_host {1e3*(t4-t3):.2f} "
          f"free {1e3*(t5-t4):.2f} total {1e3*(t5-t0):.2f} ms  groups {m}", flush=True)
