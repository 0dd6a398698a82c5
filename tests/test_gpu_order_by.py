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
