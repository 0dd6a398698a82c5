"""Diagnostic (not a test): where does a stale hipErrorInvalidDevice come from around
nut_dist calls in a torch process?  Prints hipGetLastError of the main thread after
each step."""
import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np
import torch

import nutdb_amd
from nutdb_amd import Agg, AggQuery
from nutdb_amd.dist import NutDist

hip = C.CDLL("libamdhip64.so.7")
hip.hipGetErrorName.restype = C.c_char_p


def last(tag):
    e = hip.hipGetLastError()
    d = C.c_int(-9)
    hip.hipGetDevice(C.byref(d))
    print(f"{tag:40s} lastError={e} {hip.hipGetErrorName(e).decode()} device={d.value}", flush=True)


last("start")
x = torch.ones(4, device="cuda:0")
last("after torch alloc")
n = 100000
key = torch.randint(0, 7, (n,), device="cuda:0", dtype=torch.int64)
val = torch.rand(n, device="cuda:0", dtype=torch.float64)
last("after torch randint")
for P in (2, 4, 4, 5):
    d = NutDist.virtual(P)
    last(f"virtual({P}) created")
    cuts = [(n * r // P, n * (r + 1) // P) for r in range(P)]
    qs = [AggQuery(keys=[key[a:b]], values=[val[a:b]], aggs=[Agg("sum", "col", (0,)), Agg("count")]) for a, b in cuts]
    out = d.groupby(qs, group_hint=8)
    last(f"virtual({P}) groupby")
    try:
        print(len(out[0]))
    except Exception as e:
        print("len failed:", e)
    last(f"virtual({P}) len")
    d.close()
    last(f"virtual({P}) closed")
for mk, name in ((lambda: NutDist.create([0]), "create"), (lambda: NutDist.create_rank(1, 0, NutDist.unique_id(), 0), "rank")):
    d = mk()
    last(f"{name} created")
    q = AggQuery(keys=[key], values=[val], aggs=[Agg("sum", "col", (0,)), Agg("count")])
    try:
        out = d.groupby([q], group_hint=8)
        last(f"{name} groupby")
        print(len(out[0]))
    except Exception as e:
        print("groupby failed:", e)
    last(f"{name} after")
    d.close()
    last(f"{name} closed")
print("done", flush=True)
