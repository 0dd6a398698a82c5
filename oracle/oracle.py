"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
It checks (or times, as the CPU baseline) the HIP product path; it never replaces it.
See oracle/oracle.h for the semantics and how they are pinned.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"


def build(force: bool = False) -> Path:
    src = [HERE / "oracle.c", HERE / "oracle.h"]
    if force or not LIB_PATH.exists() or any(p.stat().st_mtime > LIB_PATH.stat().st_mtime for p in src):
        subprocess.run(["make", "-s", "-C", str(HERE)] + (["-B"] if force else []), check=True)
    return LIB_PATH


class OrcAggSpec(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("nkeys", C.c_int),
        ("keys", C.c_void_p * 2),
        ("npred", C.c_int),
        ("pred_col", C.c_void_p * 6),
        ("pred_type", C.c_int * 6),
        ("pred_op", C.c_int * 6),
        ("pred_i64", C.c_int64 * 6),
        ("pred_f64", C.c_double * 6),
        ("nvals", C.c_int),
        ("val_col", C.c_void_p * 8),
        ("val_type", C.c_int * 8),
        ("naggs", C.c_int),
        ("agg_op", C.c_int * 8),
        ("agg_expr", C.c_int * 8),
        ("agg_arg", (C.c_int * 3) * 8),
        ("row_mask", C.c_void_p),
        ("agg_mask", C.c_void_p * 8),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(LIB_PATH))
        L.orc_mix64.restype = C.c_uint64
        L.orc_mix64.argtypes = [C.c_uint64]
        L.orc_gen_u64.restype = C.c_uint64
        L.orc_gen_u64.argtypes = [C.c_uint64, C.c_uint64]
        L.orc_gen_column.restype = None
        L.orc_gen_column.argtypes = [C.c_int, C.c_uint64, C.c_int64, C.c_int64, C.c_double, C.c_uint64,
                                     C.c_uint64, C.c_void_p]
        L.orc_filter_i64.restype = C.c_uint64
        L.orc_filter_i64.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int64, C.c_void_p]
        L.orc_groupby.restype = C.c_uint64
        L.orc_groupby.argtypes = [C.POINTER(OrcAggSpec), C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_groupby_tables.restype = C.c_uint64
        L.orc_groupby_tables.argtypes = [C.POINTER(OrcAggSpec), C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_join_i64.restype = C.c_uint64
        L.orc_join_i64.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p,
                                   C.c_void_p, C.c_uint64]
        L.orc_sort_i64.restype = None
        L.orc_sort_i64.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int]
        L.orc_multiset_hash_i64.restype = C.c_uint64
        L.orc_multiset_hash_i64.argtypes = [C.c_void_p, C.c_uint64]
        L.orc_max_threads.restype = C.c_int
        L.orc_eval_int.restype = C.c_int
        L.orc_eval_int.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_uint64,
                                   C.c_void_p]
        L.orc_groupby_pool_dyadic_kind.restype = C.c_uint64
        L.orc_groupby_pool_dyadic_kind.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                                   C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_groupby_pool_dyadic.restype = C.c_uint64
        L.orc_groupby_pool_dyadic.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                              C.c_void_p, C.c_void_p, C.c_int]
        _lib = L
    return _lib


F64_KINDS = (3, 4, 6)  # GEN_DYADIC, GEN_UNIT_F64, GEN_RANGE_F64


def gen_column(kind, seed, n, row0=0, a=0, b=0, c=1.0) -> np.ndarray:
    out = np.empty(n, dtype=np.float64 if kind in F64_KINDS else np.int64)
    lib().orc_gen_column(kind, seed & (2**64 - 1), a, b, c, row0, n, out.ctypes.data if n else None)
    return out


def gen(spec, n, row0=0):
    _, kind, seed, a, b, c = spec
    return gen_column(kind, seed, n, row0=row0, a=a, b=b, c=c)


def filter_i64(col: np.ndarray, op: int, k: int) -> np.ndarray:
    col = np.ascontiguousarray(col, dtype=np.int64)
    out = np.empty(max(len(col), 1), dtype=np.int64)
    cnt = lib().orc_filter_i64(col.ctypes.data, len(col), op, k, out.ctypes.data)
    return out[:cnt]


def groupby(keys, aggs, values=(), preds=(), nthreads=0, cap=None, row_mask=None, agg_masks=None,
            method="auto"):
    """keys: list of int64 arrays; values: list of arrays; preds: (array, op_int, literal);
    aggs: (op_int, expr_int, args).  row_mask / agg_masks[a]: optional bool arrays (the
    expression-mode WHERE and per-aggregate row masks, oracle/expr.py).  Returns
    (keys [n, nk] int64, words [n, na] uint64) sorted by key tuple.  method "tables" pins
    orc_groupby_tables (the per-thread-table merge; "auto" range-partitions large G with a
    bitwise-identical result)."""
    keep = []
    s = OrcAggSpec()
    if row_mask is not None:
        m = np.ascontiguousarray(row_mask, dtype=np.uint8)
        keep.append(m)
        s.row_mask = m.ctypes.data
    for a, am in enumerate(agg_masks or ()):
        if am is not None:
            m = np.ascontiguousarray(am, dtype=np.uint8)
            keep.append(m)
            s.agg_mask[a] = m.ctypes.data
    n = len(keys[0])
    s.n = n
    s.nkeys = len(keys)
    for i, k in enumerate(keys):
        k = np.ascontiguousarray(k, dtype=np.int64)
        keep.append(k)
        s.keys[i] = k.ctypes.data
    s.npred = len(preds)
    for i, (col, op, lit) in enumerate(preds):
        col = np.ascontiguousarray(col)
        keep.append(col)
        s.pred_col[i] = col.ctypes.data
        s.pred_op[i] = op
        if col.dtype == np.int64:
            s.pred_type[i] = 0
            s.pred_i64[i] = int(lit)
        else:
            s.pred_type[i] = 1
            s.pred_f64[i] = float(lit)
    s.nvals = len(values)
    for i, v in enumerate(values):
        v = np.ascontiguousarray(v)
        keep.append(v)
        s.val_col[i] = v.ctypes.data
        s.val_type[i] = 0 if v.dtype == np.int64 else 1
    s.naggs = len(aggs)
    for i, (op, ex, args) in enumerate(aggs):
        s.agg_op[i] = op
        s.agg_expr[i] = ex
        for j, x in enumerate(args):
            s.agg_arg[i][j] = x
    cap = cap if cap is not None else max(n, 1)
    ok = np.empty((cap, s.nkeys), dtype=np.int64)
    ow = np.empty((cap, max(s.naggs, 1)), dtype=np.uint64)
    fn = lib().orc_groupby_tables if method == "tables" else lib().orc_groupby
    g = fn(C.byref(s), cap, ok.ctypes.data, ow.ctypes.data, nthreads)
    if g == 2**64 - 1:
        raise ValueError("oracle group capacity too small")
    return ok[:g], ow[:g, : s.naggs]


def groupby_pool_dyadic(groups: int, n: int, row0: int = 0, key_seed: int = 0x51, val_seed: int = 0x52,
                        nthreads: int = 0, kind: int = 2):
    """Indexed oracle of the synthetic config-3 workload (oracle.h orc_groupby_pool_dyadic):
    SUM, COUNT, MIN, MAX of the dyadic value per pool key over rows [row0, row0 + n), without
    materialising the columns.  Returns (keys [m, 1] int64, words [m, 4] uint64) ordered by
    key — the layout of groupby() with aggs SUM, COUNT, MIN, MAX.  kind 7: the skewed keys
    (GEN_SKEW_KEY) of the same pool."""
    ok = np.empty((groups, 1), dtype=np.int64)
    ow = np.empty((groups, 4), dtype=np.uint64)
    m = lib().orc_groupby_pool_dyadic_kind(kind, key_seed, groups, val_seed, row0, n, ok.ctypes.data, ow.ctypes.data,
                                           nthreads)
    if m == 2**64 - 1:
        raise MemoryError("orc_groupby_pool_dyadic: allocation failed")
    return ok[:m], ow[:m]


def sort_i64(col: np.ndarray, nthreads=0) -> np.ndarray:
    col = np.ascontiguousarray(col, dtype=np.int64)
    out = np.empty_like(col)
    if len(col):
        lib().orc_sort_i64(col.ctypes.data, out.ctypes.data, len(col), nthreads)
    return out


def multiset_hash(v: np.ndarray) -> int:
    v = np.ascontiguousarray(v, dtype=np.int64)
    return int(lib().orc_multiset_hash_i64(v.ctypes.data if len(v) else None, len(v)))


def max_threads() -> int:
    return int(lib().orc_max_threads())


def join_i64(build: np.ndarray, probe: np.ndarray, how: str = "inner"):
    """Hash-join oracle (numpy, test-only): (probe_idx, build_idx) ordered by probe row,
    build rows ascending within a probe row; -1 where the join type has no build row.
    Semantics of include/nutexec.h nut_join_i64 (LEFT / SEMI / ANTI are left joins)."""
    build = np.asarray(build, dtype=np.int64)
    probe = np.asarray(probe, dtype=np.int64)
    order = np.argsort(build, kind="stable")
    sb = build[order]
    lo = np.searchsorted(sb, probe, side="left")
    hi = np.searchsorted(sb, probe, side="right")
    m = hi - lo
    rows = np.arange(len(probe), dtype=np.int64)
    if how in ("semi", "anti"):
        keep = m > 0 if how == "semi" else m == 0
        return rows[keep], np.full(int(keep.sum()), -1, dtype=np.int64)
    cnt = m if how == "inner" else np.maximum(m, 1)
    pi = np.repeat(rows, cnt)
    starts = np.repeat(lo, cnt)
    within = np.arange(len(pi), dtype=np.int64) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    bi = np.where(np.repeat(m, cnt) > 0, order[np.minimum(starts + within, len(order) - 1)] if len(order) else -1, -1)
    return pi, bi.astype(np.int64)


JOIN_TYPES = {"inner": 0, "left": 1, "semi": 2, "anti": 3}


def join_i64_c(build: np.ndarray, probe: np.ndarray, how: str = "inner"):
    """The C hash join (oracle.c orc_join_i64, OpenMP): (probe_idx, build_idx) in probe-row
    order, build rows of one probe row in unspecified order.  CPU baseline of bench.py's
    join workload; pinned against join_i64 above."""
    build = np.ascontiguousarray(build, dtype=np.int64)
    probe = np.ascontiguousarray(probe, dtype=np.int64)
    cap = len(probe)
    while True:
        pi = np.empty(max(cap, 1), dtype=np.int64)
        bi = np.empty(max(cap, 1), dtype=np.int64)
        n = lib().orc_join_i64(build.ctypes.data, len(build), probe.ctypes.data, len(probe), JOIN_TYPES[how],
                               pi.ctypes.data, bi.ctypes.data, cap)
        if n <= cap:
            return pi[:n], bi[:n]
        cap = n


def eval_int(nodes, cols, n):
    """orc_eval_int: an integer / bool RPN program (oracle/expr.py node form) over int64
    columns on every host core; None when the program is outside the C subset."""
    from .expr import OP
    ops, args, vs = [], [], []
    for node in nodes:
        op, arg, v = (tuple(node) + (0, 0))[:3]
        ops.append(OP[op] if isinstance(op, str) else int(op))
        args.append(int(arg))
        vs.append(int(v) if not isinstance(v, float) else 0)
    if any(np.asarray(c).dtype != np.int64 for c in cols):
        return None
    cols = [np.ascontiguousarray(c) for c in cols]
    ptrs = (C.c_void_p * max(len(cols), 1))(*[c.ctypes.data for c in cols])
    o, a, v = (np.asarray(x, dtype=t) for x, t in ((ops, np.int32), (args, np.int32), (vs, np.int64)))
    out = np.empty(max(n, 1), dtype=np.int64)
    r = lib().orc_eval_int(o.ctypes.data, a.ctypes.data, v.ctypes.data, len(ops), ptrs, len(cols), n, out.ctypes.data)
    return None if r else out[:n]
