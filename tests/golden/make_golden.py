"""Generate the committed golden fixtures for the executor hot path.

Independent third-party oracles, run in the build container only (numpy 2.2,
pyarrow 25, math.fsum) — the reference (nutdb v0.1.0) has no executor to run
(SURVEY.md §8(c)), so these pin the C oracle (oracle/oracle.c) and, through it and
directly, the HIP kernels.  Nothing here imports nutdb_amd or oracle/.

    python tests/golden/make_golden.py        # rewrites tests/golden/executor_golden.json

Column generator restated in numpy (uint64 arithmetic wraps mod 2^64):
    u = mix64(seed + (row + 1) * 0x9E3779B97F4A7C15)
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import numpy as np
import pyarrow as pa

OUT = Path(__file__).resolve().parent / "executor_golden.json"
U = np.uint64
GOLDEN = U(0x9E3779B97F4A7C15)
POOL_SALT = U(0x5DEECE66D2545F49)


def mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> U(30))) * U(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> U(27))) * U(0x94D049BB133111EB)
    return z ^ (z >> U(31))


def gen_u64(seed: int, n: int, row0: int = 0) -> np.ndarray:
    rows = np.arange(row0, row0 + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return mix64(U(seed) + (rows + U(1)) * GOLDEN)


def gen(kind: int, seed: int, n: int, a=0, b=0, c=1.0, row0=0) -> np.ndarray:
    u = gen_u64(seed, n, row0)
    if kind == 0:
        return (u >> U(2)).astype(np.int64)
    if kind == 1:
        return u.view(np.int64)
    if kind == 2:
        return mix64((u % U(a)) ^ POOL_SALT).view(np.int64)
    if kind == 3:
        return (u >> U(44)).astype(np.float64) / 64.0
    if kind == 4:
        return (u >> U(11)).astype(np.float64) * 2.0**-53
    if kind == 5:
        return np.int64(a) + (u % U(b)).astype(np.int64)
    if kind == 6:
        return (np.int64(a) + (u % U(b)).astype(np.int64)).astype(np.float64) / c
    raise ValueError(kind)


def wsum(v: np.ndarray) -> int:
    """wrapping uint64 sum of the raw 64-bit words"""
    with np.errstate(over="ignore"):
        return int(np.sum(v.view(np.uint64), dtype=np.uint64))


def pos_hash(v: np.ndarray) -> int:
    """order-dependent checksum: sum_i mix64(word_i + i*GOLDEN)"""
    idx = np.arange(len(v), dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int(np.sum(mix64(v.view(np.uint64) + idx * GOLDEN), dtype=np.uint64))


def multiset_hash(v: np.ndarray) -> int:
    with np.errstate(over="ignore"):
        return int(np.sum(mix64(v.view(np.uint64) ^ U(0xA0761D6478BD642F)), dtype=np.uint64))


def fhex(x: float) -> str:
    return float(x).hex()


GEN_CASES = [
    # kind, seed, a, b, c, row0
    (0, 0x2A, 0, 0, 1.0, 0),
    (1, 0x50, 0, 0, 1.0, 0),
    (2, 0x51, 1000, 0, 1.0, 0),
    (2, 0x51, 16, 0, 1.0, 123456789),
    (3, 0x52, 0, 0, 1.0, 0),
    (4, 0x52, 0, 0, 1.0, 0),
    (5, 0x41, 8036, 2526, 1.0, 0),
    (5, 0x42, 0, 3, 1.0, 0),
    (6, 0x45, 90000, 10404901, 100.0, 0),
    (6, 0x46, 0, 11, 100.0, 1000000),
]

OPS = ["<", "<=", ">", ">=", "==", "!="]


def np_cmp(col, op, k):
    return {"<": col < k, "<=": col <= k, ">": col > k, ">=": col >= k, "==": col == k, "!=": col != k}[op]


def groupby_case(G: int, dyadic: bool, n: int, pred_k=None):
    key = gen(2, 0x51, n, a=G)
    val = gen(3 if dyadic else 4, 0x52, n)
    if pred_k is not None:  # WHERE val < pred_k
        m = val < pred_k
        key, val = key[m], val[m]
    t = pa.table({"k": key, "v": val})
    r = t.group_by("k").aggregate([("v", "sum"), ("v", "count"), ("v", "min"), ("v", "max")]).sort_by("k")
    ks = r.column("k").to_numpy()
    # correctly rounded sums via fsum, per group
    order = np.argsort(key, kind="stable")
    sk, sv = key[order], val[order]
    bounds = np.flatnonzero(np.diff(sk)) + 1
    starts = np.concatenate([[0], bounds]) if len(sk) else np.array([], dtype=np.int64)
    ends = np.concatenate([bounds, [len(sk)]]) if len(sk) else np.array([], dtype=np.int64)
    fs = [math.fsum(sv[s:e]) for s, e in zip(starts, ends)]
    assert np.array_equal(sk[starts], ks)
    return {
        "G": G, "dyadic": dyadic, "n": n, "pred_val_lt": pred_k,
        "keys": [int(x) for x in ks],
        "sum_fsum": [fhex(x) for x in fs],
        "sum_arrow": [fhex(x) for x in r.column("v_sum").to_numpy()],
        "count": [int(x) for x in r.column("v_count").to_numpy()],
        "min": [fhex(x) for x in r.column("v_min").to_numpy()],
        "max": [fhex(x) for x in r.column("v_max").to_numpy()],
    }


def q1_case(n: int, date_k: int = 10471, row0: int = 0):
    sd = gen(5, 0x41, n, 8036, 2526, row0=row0)
    rf = gen(5, 0x42, n, 0, 3, row0=row0)
    ls = gen(5, 0x43, n, 0, 2, row0=row0)
    qty = gen(6, 0x44, n, 1, 50, 1.0, row0=row0)
    price = gen(6, 0x45, n, 90000, 10404901, 100.0, row0=row0)
    disc = gen(6, 0x46, n, 0, 11, 100.0, row0=row0)
    m = sd <= date_k
    t = pa.table({"rf": rf[m], "ls": ls[m], "qty": qty[m], "price": price[m],
                  "dp": price[m] * (1.0 - disc[m])})
    r = t.group_by(["rf", "ls"]).aggregate([("qty", "count")]).sort_by([("rf", "ascending"), ("ls", "ascending")])
    rows = []
    for rfv, lsv, cnt in zip(r.column("rf").to_numpy(), r.column("ls").to_numpy(), r.column("qty_count").to_numpy()):
        g = m & (rf == rfv) & (ls == lsv)
        dp = price[g] * (1.0 - disc[g])
        rows.append({
            "returnflag": int(rfv), "linestatus": int(lsv), "count": int(cnt),
            "sum_qty": fhex(math.fsum(qty[g])), "sum_price": fhex(math.fsum(price[g])),
            "sum_disc_price": fhex(math.fsum(dp)),
        })
    return {"n": n, "row0": row0, "date_k": date_k, "groups": rows}


def main():
    golden = {"generator": [], "filter": [], "groupby": [], "q1": [], "sort": []}
    n = 100_003
    for kind, seed, a, b, c, row0 in GEN_CASES:
        v = gen(kind, seed, n, a, b, c, row0)
        golden["generator"].append({
            "kind": kind, "seed": seed, "a": a, "b": b, "c": c, "row0": row0, "n": n,
            "head": [int(x) for x in v[:8].view(np.uint64)], "wsum": wsum(v),
        })
    col = gen(0, 0x2A, n)
    for s in (0.0, 0.01, 0.5, 0.9, 1.0):
        k = int(s * 2**62)
        for op in (OPS if s == 0.5 else ["<"]):
            out = col[np_cmp(col, op, k)]
            golden["filter"].append({
                "n": n, "k": k, "op": op, "count": int(len(out)),
                "head": [int(x) for x in out[:8]], "tail": [int(x) for x in out[-8:]],
                "pos_hash": pos_hash(out),
            })
    # equality on a value that exists
    kk = int(col[777])
    out = col[col == kk]
    golden["filter"].append({"n": n, "k": kk, "op": "==", "count": int(len(out)), "head": [int(x) for x in out[:8]],
                             "tail": [int(x) for x in out[-8:]], "pos_hash": pos_hash(out)})
    for G, dy in ((16, True), (1000, True), (1000, False), (5000, False)):
        golden["groupby"].append(groupby_case(G, dy, 200_003))
    golden["groupby"].append(groupby_case(1000, True, 200_003, pred_k=8000.0))
    golden["q1"].append(q1_case(300_007))
    golden["q1"].append(q1_case(65_537, row0=10**9))
    keys = gen(1, 0x50, n)
    srt = np.sort(keys)
    golden["sort"].append({"n": n, "head": [int(x) for x in srt[:8]], "tail": [int(x) for x in srt[-8:]],
                           "pos_hash": pos_hash(srt), "multiset_hash": multiset_hash(keys)})
    OUT.write_text(json.dumps(golden, indent=1) + "\n")
    print(f"wrote {OUT} ({OUT.stat().st_size} bytes)")


if __name__ == "__main__":
    main()
