"""ORDER BY with projected columns and several keys (OrderByClause.keys, reference
src/parser/ast/query.rs:86-90; the reference's fixture tests/sql/10.sql orders by a key
while projecting other columns): nut_sort_pairs (stable key + row id sort) and SQL scans
that gather their projected columns through the sorted row ids.  Parity: numpy's stable
argsort / lexsort over the same keys — row ids and gathered values bit-exact, ties in
row order (the implementation is stable; SQL allows any tie order, the test pins ours)."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

I64_MIN = np.iinfo(np.int64).min
I64_MAX = np.iinfo(np.int64).max


def dev(x, ex):
    return torch.from_numpy(np.ascontiguousarray(x)).to(ex.device)


def ukey(v, desc=False):
    """The sort's unsigned order key: int64 sign-flipped, float64 by the IEEE total order."""
    b = np.ascontiguousarray(v).view(np.uint64)
    if v.dtype == np.float64:
        u = np.where(b >> np.uint64(63), ~b, b | np.uint64(1 << 63))
    else:
        u = b ^ np.uint64(1 << 63)
    return ~u if desc else u


def sort_pairs(ex, keys, desc=False, vals=None):
    from nutdb_amd._lib import T_F64, T_I64, check, lib
    n = len(keys)
    k = dev(keys, ex)
    v = dev(vals, ex) if vals is not None else None
    out = torch.empty(max(n, 1), dtype=torch.int64, device=ex.device)
    ex._bind_stream()
    check(lib.nut_sort_pairs(ex.ctx, C.c_void_p(k.data_ptr() if n else None), T_F64 if keys.dtype == np.float64 else T_I64,
                             int(desc), C.c_void_p(v.data_ptr()) if v is not None else None,
                             C.c_void_p(out.data_ptr()), n), "nut_sort_pairs")
    ex.sync()
    return out[:n].cpu().numpy()


@pytest.mark.parametrize("n", [0, 1, 7, 8192, 8193, 100_003, 3_000_001])
@pytest.mark.parametrize("desc", [False, True])
def test_sort_pairs_i64(ex, n, desc):
    rng = np.random.default_rng(n + desc)
    keys = rng.integers(-1000, 1000, n).astype(np.int64)  # many ties: stability is visible
    if n > 10:
        keys[::11] = rng.choice(np.array([I64_MIN, I64_MAX, 0, -1], dtype=np.int64), len(keys[::11]))
    got = sort_pairs(ex, keys, desc)
    want = np.argsort(ukey(keys, desc), kind="stable")
    assert np.array_equal(got, want)


def test_sort_pairs_f64_total_order_and_payload(ex):
    rng = np.random.default_rng(5)
    n = 500_000
    keys = rng.normal(size=n)
    keys[::97] = -0.0
    keys[::89] = 0.0
    keys[::101] = np.inf
    keys[::103] = -np.inf
    keys[::107] = np.nan
    vals = rng.integers(I64_MIN, I64_MAX, n, dtype=np.int64)
    for desc in (False, True):
        got = sort_pairs(ex, keys, desc, vals)
        assert np.array_equal(got, vals[np.argsort(ukey(keys, desc), kind="stable")])


def test_sort_pairs_all_equal_and_two_keys(ex):
    keys = np.full(70_000, 42, dtype=np.int64)
    assert np.array_equal(sort_pairs(ex, keys), np.arange(70_000))
    # two keys the LSD way: the least significant first, its order as the next payload
    rng = np.random.default_rng(6)
    a = rng.integers(0, 50, 200_000).astype(np.int64)
    b = rng.normal(size=200_000)
    p = sort_pairs(ex, b, desc=True)
    p = sort_pairs(ex, a[p], vals=p)
    assert np.array_equal(p, np.lexsort((ukey(b, True), ukey(a))))


def _table(n, seed):
    rng = np.random.default_rng(seed)
    return {"a": rng.integers(-50, 50, n).astype(np.int64), "b": rng.integers(0, 7, n).astype(np.int64),
            "c": rng.normal(size=n), "d": rng.integers(I64_MIN, I64_MAX, n, dtype=np.int64)}


@pytest.mark.parametrize("sql, keys, where, lim", [
    ("select a, c, d from t order by b desc, a", [("b", True), ("a", False)], None, None),
    ("select d, a from t where a > 10 order by c", [("c", False)], lambda t: t["a"] > 10, None),
    ("select c as cc, b from t where b <> 3 order by cc desc, b limit 1000 offset 17",
     [("c", True), ("b", False)], lambda t: t["b"] != 3, (1000, 17)),
    ("select a from t order by b, c desc, d", [("b", False), ("c", True), ("d", False)], None, None),
    ("select b, d from t where a < -40 or a > 45 order by d desc limit 5", [("d", True)],
     lambda t: (t["a"] < -40) | (t["a"] > 45), (5, 0)),
])
def test_sql_order_by_projected_columns(ex, sql, keys, where, lim):
    from nutdb_amd.sql import Plan
    n = 1_000_003
    t = _table(n, 7)
    got = Plan(sql).execute(ex, {k: dev(v, ex) for k, v in t.items()})
    ids = np.nonzero(where(t))[0] if where else np.arange(n)
    order = ids[np.lexsort(tuple(ukey(t[k][ids], d) for k, d in reversed(keys)))]
    if lim:
        order = order[lim[1]:lim[1] + lim[0]]
    proj = sql.split(" from ")[0][len("select "):].split(", ")
    for item in proj:
        col, _, alias = item.partition(" as ")
        name = alias or col
        assert np.array_equal(got[name].view(np.uint64), t[col][order].view(np.uint64)), name


def test_sql_order_by_fixture10_shape_typed_table(ex):
    """The reference fixture tests/sql/10.sql orders employees by e.employee_id while
    projecting other columns (strings included): the same shape over a typed table."""
    from nutdb_amd.sql import Plan
    from nutdb_amd.table import Table
    t = Table(ex, "CREATE TABLE employees (employee_id Int64, first_name String, email String, "
                  "commission_pct Float64, job_id Int32)")
    rng = np.random.default_rng(3)
    n = 20_000
    ids = rng.permutation(n).astype(np.int64) + 100
    first = [f"name{i % 977}" for i in range(n)]
    email = [f"e{i}@x" for i in range(n)]
    pct = rng.random(n)
    job = rng.integers(1, 20, n).astype(np.int32)
    t.append(employee_id=ids, first_name=first, email=email, commission_pct=pct, job_id=job)
    got = t.execute(Plan("SELECT employee_id AS `Employee #`, first_name AS Name, email AS Email, "
                             "commission_pct AS `Comission %` FROM employees WHERE job_id > 3 "
                             "ORDER BY employee_id"))
    sel = np.nonzero(job > 3)[0]
    order = sel[np.argsort(ids[sel], kind="stable")]
    assert np.array_equal(got["Employee #"], ids[order])
    assert list(got["Name"]) == [first[i] for i in order]
    assert list(got["Email"]) == [email[i] for i in order]
    assert np.array_equal(got["Comission %"], pct[order])


def test_sql_order_by_string_key_rejected(ex):
    from nutdb_amd import NutError
    from nutdb_amd.sql import Plan
    from nutdb_amd.table import Table
    t = Table(ex, "CREATE TABLE e (id Int64, name String)")
    t.append(id=np.arange(10, dtype=np.int64), name=[str(i) for i in range(10)])
    with pytest.raises(NutError, match="string column"):
        t.execute(Plan("SELECT id FROM e ORDER BY name"))


# ------------------------------------------------------------------ ORDER BY ... LIMIT (top-k)
def topk_positions(ex, keys, k, desc=False, cap=None):
    from nutdb_amd._lib import T_F64, T_I64, lib
    n = len(keys)
    d = dev(keys, ex)
    cap = n if cap is None else cap
    out = torch.empty(max(cap, 1), dtype=torch.int64, device=ex.device)
    cnt = C.c_uint64()
    ex._bind_stream()
    st = lib.nut_topk_positions(ex.ctx, C.c_void_p(d.data_ptr()), T_F64 if keys.dtype == np.float64 else T_I64,
                                1 if desc else 0, n, k, C.c_void_p(out.data_ptr()), cap, C.byref(cnt))
    ex.sync()
    return st, cnt.value, out[: cnt.value].cpu().numpy()


@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("kind", ["uniform", "narrow", "ties", "f64"])
def test_topk_positions(ex, kind, desc):
    """nut_topk_positions: ascending positions of every key ordered at or before the k-th
    (ties included), at least k of them — exactly the keys u <= the k-th key's u plus the
    rest of its final radix bucket; checked against numpy on the order-mapped keys."""
    rng = np.random.default_rng(91)
    n = 3_000_017
    keys = {"uniform": lambda: rng.integers(I64_MIN, I64_MAX, n, dtype=np.int64),
            "narrow": lambda: rng.integers(-5000, 5000, n).astype(np.int64),
            "ties": lambda: np.repeat(rng.integers(0, 40, n // 100 + 1), 100)[:n].astype(np.int64),
            "f64": lambda: np.where(rng.random(n) < 0.01, -0.0, rng.standard_normal(n))}[kind]()
    u = ukey(keys, desc)
    su = np.sort(u)
    for k in (1, 10, 1000, 250_000, n - 1, n, n + 5):
        st, cnt, pos = topk_positions(ex, keys, k, desc)
        assert st == 0, (k, st)
        kth = su[min(k, n) - 1]
        assert cnt >= min(k, n) and np.all(np.diff(pos) > 0)
        assert np.array_equal(np.sort(pos), pos)
        inside = u[pos]
        assert np.all(inside <= inside.max()) and int((u <= kth).sum()) <= cnt  # every tie of the k-th key
        assert np.array_equal(pos, np.flatnonzero(u <= inside.max())), k  # a prefix of the order
    # capacity: reported, nothing written
    st, cnt, _ = topk_positions(ex, keys, 1000, desc, cap=10)
    assert st == 5 and cnt >= 1000


@pytest.mark.parametrize("topk", [1, 0])
def test_sql_order_by_limit_topk(ex, opts, topk):
    """ORDER BY ... LIMIT runs a stable sort of only the top-k candidate rows; results are
    identical to the full sort (option topk=0) and to numpy's stable order, ties in row
    order — keys-only scans (fused and expression mode), projected columns with several
    keys, DESC, float64 keys, OFFSET, heavy ties at the boundary, and LIMIT 0."""
    opts(topk=topk)
    rng = np.random.default_rng(13)
    n = 2_000_003
    a = rng.integers(-10**6, 10**6, n).astype(np.int64)
    b = rng.integers(0, 50, n).astype(np.int64)  # heavy ties
    f = rng.standard_normal(n)
    cols = {"a": dev(a, ex), "b": dev(b, ex), "f": dev(f, ex)}
    # keys-only, fused (no WHERE / one comparison of the column) and expression mode
    got = ex.sql("select a from t order by a limit 100", cols)["a"]
    assert np.array_equal(got, np.sort(a)[:100])
    got = ex.sql("select a from t where a > 5 order by a desc limit 37 offset 11", cols)["a"]
    assert np.array_equal(got, np.sort(a[a > 5])[::-1][11:48])
    got = ex.sql("select a from t where a % 3 = 0 order by a limit 1000", cols)["a"]
    assert np.array_equal(got, np.sort(a[a % 3 == 0])[:1000])
    # projected columns, several keys, ties broken by the next key then by row order
    got = ex.sql("select a, b, f from t where b < 45 order by b, a desc limit 500 offset 3", cols)
    idx = np.flatnonzero(b < 45)
    o = idx[np.lexsort((-a[idx], b[idx]))][3:503]
    assert np.array_equal(got["b"], b[o]) and np.array_equal(got["a"], a[o]) and np.array_equal(got["f"], f[o])
    # a float64 key (IEEE total order), DESC
    got = ex.sql("select f, a from t order by f desc limit 64", cols)
    o = np.argsort(ukey(f, desc=True), kind="stable")[:64]
    assert np.array_equal(got["f"], f[o]) and np.array_equal(got["a"], a[o])
    # the boundary key repeats ~40000 times: every tie is a candidate
    got = ex.sql("select b, a from t order by b limit 70000", cols)
    o = np.argsort(b, kind="stable")[:70000]
    assert np.array_equal(got["b"], b[o]) and np.array_equal(got["a"], a[o])
    assert len(ex.sql("select a from t order by a limit 0", cols)["a"]) == 0
