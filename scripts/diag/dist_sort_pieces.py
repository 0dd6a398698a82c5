"""Diagnostic: which piece of the single-rank dist sort breaks at 2e8 keys."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from nutdb_amd import Executor  # noqa: E402
from nutdb_amd.dist import NutDist  # noqa: E402
from nutdb_amd.workloads import SORT_COL, gen  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000_000
ex = Executor(0)
col = gen(ex, SORT_COL, n)
ref = ex.sort_i64(col)
print("single", ex.sort_stats(), flush=True)
part, counts = ex.partition_i64(col, [])
print("partition nsplit=0 equal input:", bool(torch.equal(part, col)), counts, flush=True)
s2 = ex.sort_i64(part)
print("sort of partition output equal:", bool(torch.equal(s2, ref)), ex.sort_stats(), flush=True)
for mk in ("virtual", "rank"):
    nd = NutDist.virtual(1) if mk == "virtual" else NutDist.create_rank(1, 0, NutDist.unique_id(), 0)
    out = nd.sort_i64([col])[0]
    print(mk, "dist sort equal:", bool(torch.equal(out, ref)), nd.sort_stats(), flush=True)
    nd.close()
