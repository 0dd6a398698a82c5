"""Diagnostic: virtual P-rank sample sort of P x n keys (one GPU), for a kernel trace of the
per-rank partition / local sort; checks the result (sorted ranks, multiset)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from nutdb_amd import Executor  # noqa: E402
from nutdb_amd.dist import NutDist  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 1.5e8
ex = Executor(0)
keys = ex.gen_column(1, 0x77, P * n)
torch.cuda.synchronize()
d = NutDist.virtual(P)
for rep in range(2):
    outs = d.sort_i64([keys[r * n:(r + 1) * n] for r in range(P)], copy=False)
sizes = [c for _, c in outs]
stats = [d.sort_stats(l) for l in range(P)]
print("P", P, "n/rank", n, "received", sizes, "bytes/key", [round(b / max(c, 1), 1) for (b, _), c in zip(stats, sizes)])
d.close()
