"""Diagnostic: SEMI / ANTI steps of a join chain (EXISTS / IN subqueries) vs a single
LEFT SEMI JOIN and the raw join."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from nutdb_amd import Executor  # noqa: E402

ex = Executor(0)
rng = np.random.default_rng(1)
t = {"k": rng.integers(0, 2000, 5000).astype(np.int64), "x": rng.integers(0, 100, 5000).astype(np.int64)}
u = {"uk": rng.integers(0, 2000, 8000).astype(np.int64), "w": rng.integers(0, 10, 8000).astype(np.int64)}
d = lambda c: {k: torch.from_numpy(v).cuda() for k, v in c.items()}  # noqa: E731
want = int(np.isin(t["k"], u["uk"]).sum())
pi, bi = ex.join_i64(d(u)["uk"], d(t)["k"], how="semi")
print("raw semi join pairs", len(pi), "want", want, flush=True)
r = ex.sql("select count(*) as c from t left semi join u on k = uk", d(t), right=d(u))
print("single LEFT SEMI JOIN", r["c"], flush=True)
r = ex.sql("select count(*) as c from t where k in (select uk from u)", d(t), right=[d(u)])
print("IN subquery (no filter)", r["c"], flush=True)
r = ex.sql("select count(*) as c from t where exists (select * from u where uk = k)", d(t), right=[d(u)])
print("EXISTS (no filter)", r["c"], flush=True)
want7 = int(np.isin(t["k"], u["uk"][u["w"] < 7]).sum())
r = ex.sql("select count(*) as c from t where k in (select uk from u where w < 7)", d(t), right=[d(u)])
print("IN subquery (w < 7)", r["c"], "want", want7, flush=True)
r = ex.sql("select k from t where k in (select uk from u where w < 7)", d(t), right=[d(u)])
print("IN scan rows", len(r["k"]), "want", want7, flush=True)
