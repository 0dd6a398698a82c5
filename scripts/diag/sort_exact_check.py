"""Diagnostic: where does a sort of range-restricted keys with two outliers go wrong?"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from nutdb_amd import Executor  # noqa: E402

ex = Executor(0)


def run(n, lo, width, outliers, tag):
    keys = ex.gen_column(5, 0x42, n, a=lo, b=width)
    if outliers:
        keys[n // 2 + 3] = -(2**63)
        keys[n // 3 + 5] = 2**63 - 1
    out = ex.sort_i64(keys)
    st = ex.sort_stats()
    o = out.cpu().numpy()
    want = np.sort(keys.cpu().numpy())
    bad = np.nonzero(o != want)[0]
    print(tag, "n", n, "stats", st, "bytes/key", st[0] / n, "wrong", len(bad), flush=True)
    if len(bad):
        f = bad[0]
        print("   first wrong", f, "last", bad[-1], "got", o[f:f + 4], "want", want[f:f + 4], flush=True)
        # runs of wrong positions
        br = np.nonzero(np.diff(bad) != 1)[0]
        print("   runs", len(br) + 1, "first runs", [(int(bad[0]), int(bad[br[0]]) if len(br) else int(bad[-1]))], flush=True)


run(1 << 22, 1 << 50, 1 << 52, True, "exact small + outliers")
run(1 << 24, 1 << 50, 1 << 52, True, "exact 2^24 + outliers")
run(1 << 24, 1 << 50, 1 << 52, False, "exact 2^24 narrow")
run((1 << 26) + 12345, 1 << 50, 1 << 52, False, "capped 2^26 narrow")
run((1 << 26) + 12345, 1 << 50, 1 << 52, True, "2^26 + outliers")
run((1 << 26) + 12345, -(2**62), 2**63 - 1, True, "2^26 wide + outliers")
run((1 << 26) + 12345, -(2**63), 2**63 - 1, False, "2^26 half range")
