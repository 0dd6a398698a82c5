"""Diagnostic: the test_gpu_sort_range sequence on one context, repeated; reports where an
output differs from np.sort."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from nutdb_amd import Executor  # noqa: E402

ex = Executor(0)
N = (1 << 26) + 12345


def check(tag, keys, desc=False, outl=False):
    out = ex.sort_i64(keys, descending=desc)
    st = ex.sort_stats()
    o = out.cpu().numpy()
    want = np.sort(keys.cpu().numpy())
    if desc:
        want = want[::-1]
    bad = np.nonzero(o != want)[0]
    print(tag, "bytes/key %.2f" % (st[0] / len(o)), "levels", st[1], "wrong", len(bad), flush=True)
    if len(bad):
        f = bad[0]
        print("   first", f, "last", bad[-1], "got", o[f:f + 3], "want", want[f:f + 3], flush=True)
        br = np.nonzero(np.diff(bad) != 1)[0]
        print("   runs", len(br) + 1, "lens", np.diff(np.concatenate([[-1], br, [len(bad) - 1]]))[:10], flush=True)


for rep in range(3):
    for lo, width in [(3 << 60, 1 << 61), (-(1 << 62) + 12345, 3_000_000_000_007), (-(1 << 40), (1 << 41) + 1),
                      (10**15, 1 << 30)]:
        for desc in (False, True):
            check(f"r{rep} range {lo} {width} desc={desc}", ex.gen_column(5, 0x77 + width % 1000, N, a=lo, b=width), desc)
    keys = ex.gen_column(5, 0x42, N, a=1 << 50, b=1 << 52)
    keys[N // 2 + 3] = -(2**63)
    keys[N // 3 + 5] = 2**63 - 1
    check(f"r{rep} outliers", keys)
    check(f"r{rep} narrow", ex.gen_column(5, 0x43, N, a=-5, b=1 << 20))
