"""UNION ALL on the GPU, against pandas.

The reference's fixture tests/sql/12.sql is a CREATE VIEW whose body is a UNION ALL of four
scans (SUPPLY1 with a WHERE, SUPPLY2..4 without).  The executor plans the view's body: every
branch is its own single-table plan, run in branch order over its own table
(nut_plan_executen / nut_table_executen: branch k over table k), and the results are
concatenated on the device (scans) or the host (aggregates), decoded strings and NULL flags
per branch.  Row order = branch order, then each branch's own order."""
import numpy as np
import pandas as pd
import pytest
import torch

from nutdb_amd.sql import Plan
from nutdb_amd.table import Table

pytestmark = pytest.mark.gpu

FIXTURE12 = open(__file__.rsplit("/", 1)[0] + "/golden/sql/12.sql").read()


def on_dev(ex, cols):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(ex.device) for k, v in cols.items()}


def supply(rng, n, sth=False):
    t = {"supplyID": rng.integers(0, 10_000, n).astype(np.int64), "supplier": rng.integers(-50, 50, n).astype(np.int64)}
    if sth:
        t["sth"] = rng.integers(0, 3, n).astype(np.int64)
    return t


def test_fixture12_view_body_raw_columns(ex):
    rng = np.random.default_rng(12)
    tabs = [supply(rng, 1_000_003, sth=True), supply(rng, 77), supply(rng, 0), supply(rng, 250_000)]
    got = Plan(FIXTURE12).execute_tables(ex, [on_dev(ex, t) for t in tabs])
    parts = [pd.DataFrame(tabs[0])[tabs[0]["sth"] == 1][["supplyID", "supplier"]]]
    parts += [pd.DataFrame(t)[["supplyID", "supplier"]] for t in tabs[1:]]
    want = pd.concat(parts)
    assert list(got) == ["supplyID", "supplier"]
    assert np.array_equal(got["supplyID"], want["supplyID"].to_numpy())
    assert np.array_equal(got["supplier"], want["supplier"].to_numpy())


def test_fixture12_view_body_typed_tables_with_strings(ex):
    """The same view over typed tables whose `supplier` is a String column: each table has
    its own dictionary, and the concatenated result decodes every branch with its own."""
    rng = np.random.default_rng(21)
    names = np.array([f"supplier#{i:05d}" for i in range(300)], dtype=object)
    tabs, data = [], []
    for k in range(4):
        n = [40_000, 1_000, 5, 123_456][k]
        cols = {"supplyID": rng.integers(0, 1000, n).astype(np.int64), "supplier": rng.choice(names[k * 50:k * 50 + 120], n)}
        ddl = "CREATE TABLE SUPPLY%d (supplyID Int64, supplier String%s)" % (k + 1, ", sth Int8" if k == 0 else "")
        if k == 0:
            cols["sth"] = rng.integers(0, 2, n).astype(np.int8)
        t = Table(ex, ddl)
        t.append(**cols)
        tabs.append(t)
        data.append(cols)
    got = tabs[0].execute_joins(Plan(FIXTURE12), tabs[1:])
    d0 = pd.DataFrame(data[0])
    want = pd.concat([d0[d0["sth"] == 1][["supplyID", "supplier"]]] +
                     [pd.DataFrame(c)[["supplyID", "supplier"]] for c in data[1:]])
    assert np.array_equal(got["supplyID"], want["supplyID"].to_numpy())
    assert list(got["supplier"]) == list(want["supplier"])


def test_union_all_one_table_expressions_and_nulls(ex):
    """Every branch over the same columns (nut_plan_execute): computed projections, a CASE
    without ELSE (NULL flags in one branch only), an ORDER BY ... LIMIT inside a branch."""
    rng = np.random.default_rng(5)
    n = 200_000
    a = rng.integers(-1000, 1000, n).astype(np.int64)
    b = rng.integers(0, 100, n).astype(np.int64)
    sql = ("select a * 2 as x, case when b < 50 then b end as y from t where a > 900 "
           "union all select a, b from t where b = 7 "
           "union all select a, b from t where a < -990 order by a desc limit 5")
    got = Plan(sql).execute(ex, on_dev(ex, {"a": a, "b": b}))
    m0, m1 = a > 900, b == 7
    top = np.sort(a[a < -990])[::-1][:5]
    x = np.concatenate([a[m0] * 2, a[m1], top])
    assert np.array_equal(np.asarray(got["x"]), x)
    y = got["y"]
    assert isinstance(y, np.ma.MaskedArray)
    y0 = np.where(b[m0] < 50, b[m0], -1)
    want_mask = np.concatenate([b[m0] >= 50, np.zeros(m1.sum() + len(top), bool)])
    assert np.array_equal(np.ma.getmaskarray(y), want_mask)
    assert np.array_equal(np.asarray(y)[:m0.sum()][b[m0] < 50], y0[b[m0] < 50])
    assert np.array_equal(np.asarray(y)[m0.sum():m0.sum() + m1.sum()], b[m1])


def test_union_all_of_aggregates(ex):
    rng = np.random.default_rng(9)
    t1 = {"k": rng.integers(0, 50, 300_000).astype(np.int64), "v": rng.random(300_000)}
    t2 = {"k": rng.integers(100, 130, 100_000).astype(np.int64), "v": rng.random(100_000)}
    sql = ("select k, count(*) as n, sum(v) as s from t1 group by k order by k "
           "union all select k, count(*), sum(v) from t2 group by k order by k")
    got = Plan(sql).execute_tables(ex, [on_dev(ex, t1), on_dev(ex, t2)])
    want = pd.concat([pd.DataFrame(t).groupby("k").agg(n=("v", "size"), s=("v", "sum")).reset_index() for t in (t1, t2)])
    assert np.array_equal(got["k"], want["k"].to_numpy()) and np.array_equal(got["n"], want["n"].to_numpy())
    assert np.allclose(got["s"], want["s"].to_numpy(), rtol=1e-12, atol=0)


@pytest.mark.parametrize("sql", ["select a from t union all select f from u",
                                 "select sum(a) from t union all select sum(f) from u"])
def test_union_all_type_mismatch_is_a_plan_error(ex, sql):
    from nutdb_amd import NutError
    a = torch.arange(10, dtype=torch.int64, device=ex.device)
    f = torch.arange(10, dtype=torch.float64, device=ex.device)
    with pytest.raises(NutError, match="UNION ALL: column 1"):
        Plan(sql).execute_tables(ex, [{"a": a}, {"f": f}])
