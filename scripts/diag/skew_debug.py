"""Which groups of the ordered Zipf-key group-by differ from the oracle (heavy pass on)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from nutdb_amd import Executor, _lib as L  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from test_gpu_exec import gb_query  # noqa: E402

ex = Executor()
N = (1 << 24) + 4099
G = 4_000_000
key = ex.gen_column(L.GEN_SKEW_KEY, 0x51, N, a=G)
val = ex.gen_column(L.GEN_DYADIC, 0x52, N)
q = gb_query(key, val)
ok, ow = orc.groupby_pool_dyadic(G, N, key_seed=0x51, val_seed=0x52, kind=7)
hint = ok.shape[0]
for heavy in (1, 0):
    ex.set_option("gb_heavy", heavy)
    out = tuple(torch.empty((2 * hint, w), dtype=torch.int64, pin_memory=True).numpy() for w in (1, 4))
    k, w = ex.groupby_to_host(q, group_hint=hint, out=out)
    k, w = k.copy(), w.copy().view(np.uint64)
    print("heavy", heavy, "path", ex.groupby_stats()["path"], "heavy", ex.groupby_heavy(),
          "overflow", ex.groupby_overflow_rows(), "groups", len(k), "want", len(ok), flush=True)
    if len(k) != len(ok) or not np.array_equal(k, ok):
        print("  keys differ", flush=True)
        continue
    bad = np.nonzero((w != ow).any(axis=1))[0]
    print("  rows differing:", len(bad), flush=True)
    for i in bad[:10]:
        print("   key", int(k[i, 0]), "got", [int(x) for x in w[i]], "want", [int(x) for x in ow[i]],
              "count ratio", int(w[i, 1]) / max(1, int(ow[i, 1])), flush=True)
