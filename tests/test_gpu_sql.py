"""GPU: SQL text -> nut_sql_plan -> HIP kernels, checked against the C oracle / numpy.

Covers the plan lowering row end to end: the TPC-H Q1 text of the
reference's fixture family (toDate/interval constants, fused expressions, avg), the
filter / sort / group-by plan kinds, constant-comparison folding against int64 columns,
ORDER BY / LIMIT over group results, and the binding errors.
Tolerances: integer results bit-exact; f64 sums of non-dyadic values <= 1e-12 relative.
"""
import numpy as np
import pytest
import torch

from helpers import F64_SUM_RTOL, OPCODE, rel_err

pytestmark = pytest.mark.gpu

LINEITEM_TAX = ("l_tax", 6, 0x47, 0, 9, 100.0)  # RANGE_F64: 0.00..0.08


def dev(x, ex):
    return torch.from_numpy(np.ascontiguousarray(x)).to(ex.device)


def test_sql_tpch_q1(ex, orc):
    from nutdb_amd.workloads import Q1_COLS, gen
    n = 2_000_003
    specs = Q1_COLS + [LINEITEM_TAX]
    cols = {s[0]: gen(ex, s, n) for s in specs}
    sql = """select l_returnflag, l_linestatus, sum(l_quantity) as sum_qty, sum(l_extendedprice) as sum_base_price,
        sum(l_extendedprice * (1 - l_discount)) as sum_disc_price,
        sum(l_extendedprice * (1 - l_discount) * (1 + l_tax)) as sum_charge,
        avg(l_quantity) as avg_qty, avg(l_extendedprice) as avg_price, avg(l_discount) as avg_disc,
        count(*) as count_order
      from lineitem
      where l_shipdate <= toDate('1998-12-01') - interval 90 day
      group by l_returnflag, l_linestatus
      order by l_returnflag, l_linestatus"""
    got = ex.sql(sql, cols, group_hint=6)
    sd, rf, ls, qty, price, disc, tax = [orc.gen(s, n) for s in specs]
    ok, ow = orc.groupby([rf, ls], [(0, 0, (0,)), (0, 0, (1,)), (0, 4, (1, 2)), (0, 5, (1, 2, 3)), (1, 0, ()),
                                    (0, 0, (2,))],
                         values=[qty, price, disc, tax], preds=[(sd, OPCODE["<="], 10471)])
    f = ow.view(np.float64)
    cnt = ow[:, 4].astype(np.int64)
    assert list(got) == ["l_returnflag", "l_linestatus", "sum_qty", "sum_base_price", "sum_disc_price",
                         "sum_charge", "avg_qty", "avg_price", "avg_disc", "count_order"]
    assert np.array_equal(got["l_returnflag"], ok[:, 0]) and np.array_equal(got["l_linestatus"], ok[:, 1])
    assert np.array_equal(got["count_order"], cnt)
    for name, j in (("sum_qty", 0), ("sum_base_price", 1), ("sum_disc_price", 2), ("sum_charge", 3)):
        assert rel_err(got[name], f[:, j]) <= F64_SUM_RTOL, name
    for name, j in (("avg_qty", 0), ("avg_price", 1), ("avg_disc", 5)):
        assert rel_err(got[name], f[:, j] / cnt) <= 2 * F64_SUM_RTOL, name


def test_sql_filter_plans(ex, orc):
    from nutdb_amd.workloads import FILTER_COL, filter_k, gen
    n = 3_000_017
    col = gen(ex, FILTER_COL, n)
    h = orc.gen(FILTER_COL, n)
    k = filter_k(0.3)
    want = orc.filter_i64(h, OPCODE["<"], k)
    t = {"col": col}
    assert np.array_equal(ex.sql(f"select col from t where col < {k}", t)["col"], want)
    assert np.array_equal(ex.sql(f"select col from t where {k} > col", t)["col"], want)
    # a non-integral constant moves the bound: col <= k.5  ==  col <= k
    assert np.array_equal(ex.sql(f"select col from t where col <= {k}.5", t)["col"], h[h <= k])
    assert np.array_equal(ex.sql(f"select col from t where col >= {k}.5", t)["col"], h[h > k])
    # constants outside int64 fold to all/none
    assert len(ex.sql("select col from t where col < 99999999999999999999999", t)["col"]) == n
    assert len(ex.sql("select col from t where col > -1.5", t)["col"]) == n
    assert len(ex.sql("select col from t where col = 3.5", t)["col"]) == 0
    assert len(ex.sql("select col from t where 1 = 0", t)["col"]) == 0
    assert np.array_equal(ex.sql("select col from t", t)["col"], h)
    got = ex.sql(f"select col as c from t where col < {k} limit 10 offset 5", t)
    assert list(got) == ["c"] and np.array_equal(got["c"], want[5:15])


def test_sql_sort_plans(ex, orc):
    from nutdb_amd.workloads import SORT_COL, gen
    n = 1_000_003
    key = gen(ex, SORT_COL, n)
    h = orc.gen(SORT_COL, n)
    s = np.sort(h)
    t = {"k": key}
    assert np.array_equal(ex.sql("select k from t order by k", t)["k"], s)
    assert np.array_equal(ex.sql("select k from t order by k desc", t)["k"], s[::-1])
    assert np.array_equal(ex.sql("select k from t where k < 0 order by k desc limit 100", t)["k"],
                          np.sort(h[h < 0])[::-1][:100])
    # direct descending entry point, including duplicates and extremes
    v = np.concatenate([h[:1000], np.repeat(h[:10], 50), [np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0, -1]])
    out = ex.sort_i64(dev(v, ex), descending=True).cpu().numpy()
    assert np.array_equal(out, np.sort(v)[::-1])


def test_sql_groupby_order_limit(ex, orc):
    from nutdb_amd import _lib as L
    n = 1_500_007
    G = 50
    kspec = ("k", L.GEN_POOL_KEY, 0x61, G, 0, 1.0)
    vspec = ("v", L.GEN_DYADIC, 0x62, 0, 0, 1.0)
    ispec = ("i", L.GEN_FULL_I64, 0x63, 0, 0, 1.0)
    cols = {s[0]: ex.gen_column(s[1], s[2], n, a=s[3], b=s[4], c=s[5]) for s in (kspec, vspec, ispec)}
    k, v, i = (orc.gen(s, n) for s in (kspec, vspec, ispec))
    got = ex.sql("select k, sum(v) as s, count(*) as c, min(v), max(v), avg(v) as a, sum(i) as si from t "
                 "where v > 0.25 and v <= 8000 group by k order by c desc, k limit 7 offset 2", cols)
    m = (v > 0.25) & (v <= 8000)
    uk, inv = np.unique(k[m], return_inverse=True)
    cnt = np.bincount(inv)
    sums = np.bincount(inv, weights=v[m])  # dyadic values: exact in any order
    mins = np.full(len(uk), np.inf)
    maxs = np.full(len(uk), -np.inf)
    np.minimum.at(mins, inv, v[m])
    np.maximum.at(maxs, inv, v[m])
    isum = np.zeros(len(uk), dtype=np.uint64)
    np.add.at(isum, inv, i[m].view(np.uint64))  # two's-complement wrap
    order = np.lexsort((uk, -cnt))[2:9]
    assert list(got) == ["k", "s", "c", "min(v)", "max(v)", "a", "si"]
    assert np.array_equal(got["k"], uk[order])
    assert np.array_equal(got["c"], cnt[order])
    assert np.array_equal(got["s"], sums[order])
    assert np.array_equal(got["min(v)"], mins[order]) and np.array_equal(got["max(v)"], maxs[order])
    assert np.array_equal(got["a"], sums[order] / cnt[order])
    assert np.array_equal(got["si"], isum[order].view(np.int64))


def test_sql_binding_errors(ex):
    from nutdb_amd import NutError
    a = torch.zeros(10, dtype=torch.int64, device=ex.device)
    with pytest.raises(NutError) as e:
        ex.sql("select k, sum(v) from t group by k", {"k": a})
    assert e.value.status == 1 and "'v' is not bound" in str(e.value)
    with pytest.raises(NutError) as e:
        ex.sql("select k, sum(v * w) from t group by k", {"k": a, "v": a, "w": a})
    assert e.value.status == 7 and "float64" in str(e.value)
    # a Float64 GROUP BY column groups on its key words: no longer an error
    got = ex.sql("select k from t group by k", {"k": a.double()})
    assert got["k"].dtype == np.float64 and list(got["k"]) == [0.0]
    with pytest.raises(NutError) as e:  # a computed Float64 key still is
        ex.sql("select k * 2 as j from t group by j", {"k": a.double()})
    assert e.value.status == 7 and "float64" in str(e.value)


def test_sql_tpch_q6_global_aggregate(ex, orc):
    """TPC-H Q6: five predicates (BETWEEN + date interval) and SUM(a*b) without GROUP BY."""
    import math
    from nutdb_amd.workloads import Q1_COLS, gen
    n = 3_000_001
    cols = {s[0]: gen(ex, s, n) for s in Q1_COLS}
    got = ex.sql("""select sum(l_extendedprice * l_discount) as revenue, count(*) as n from lineitem
        where l_shipdate >= toDate('1994-01-01') and l_shipdate < toDate('1994-01-01') + interval 1 year
          and l_discount between 0.05 and 0.07 and l_quantity < 24""", cols)
    sd, _, _, qty, price, disc = [orc.gen(s, n) for s in Q1_COLS]
    m = (sd >= 8766) & (sd < 9131) & (disc >= 0.05) & (disc <= 0.07) & (qty < 24)
    assert list(got) == ["revenue", "n"]
    assert got["n"].tolist() == [int(m.sum())]
    want = math.fsum((price[m] * disc[m]).tolist())
    assert rel_err(got["revenue"], [want]) <= F64_SUM_RTOL


def test_sql_global_aggregates_and_empty(ex):
    rng = np.random.default_rng(11)
    n = 1_000_003
    v = rng.integers(0, 1 << 20, n) / 64.0  # dyadic: exact sums
    i = rng.integers(-1000, 1000, n).astype(np.int64)
    t = {"v": dev(v, ex), "i": dev(i, ex)}
    got = ex.sql("select count(*), sum(v), min(v), max(v), avg(v), sum(i), min(i) from t where v > 4096", t)
    m = v > 4096
    assert got["count(*)"].tolist() == [int(m.sum())]
    assert got["sum(v)"].tolist() == [float(v[m].sum())]
    assert got["min(v)"].tolist() == [float(v[m].min())] and got["max(v)"].tolist() == [float(v[m].max())]
    assert got["avg(v)"].tolist() == [float(v[m].sum()) / int(m.sum())]
    assert got["sum(i)"].tolist() == [int(i[m].sum())] and got["min(i)"].tolist() == [int(i[m].min())]
    empty = ex.sql("select count(*), sum(v), avg(v) from t where 1 = 0", t)
    assert empty["count(*)"].tolist() == [0] and empty["sum(v)"].tolist() == [0.0]
    assert np.isnan(empty["avg(v)"][0])


def test_sql_having_and_order_by_aggregate(ex, orc):
    from nutdb_amd import _lib as L
    n = 1_200_007
    kspec = ("k", L.GEN_POOL_KEY, 0x71, 300, 0, 1.0)
    vspec = ("v", L.GEN_DYADIC, 0x72, 0, 0, 1.0)
    cols = {s[0]: ex.gen_column(s[1], s[2], n, a=s[3], b=s[4], c=s[5]) for s in (kspec, vspec)}
    k, v = (orc.gen(s, n) for s in (kspec, vspec))
    got = ex.sql("select k, sum(v) as s from t group by k having count(*) >= 4000 and not (s < 32000000) "
                 "or k between -10 and 10 order by max(v) desc, k", cols, group_hint=300)
    uk, inv = np.unique(k, return_inverse=True)
    cnt = np.bincount(inv)
    sums = np.bincount(inv, weights=v)
    maxs = np.full(len(uk), -np.inf)
    np.maximum.at(maxs, inv, v)
    keep = ((cnt >= 4000) & ~(sums < 32000000)) | ((uk >= -10) & (uk <= 10))
    order = np.lexsort((uk[keep], -maxs[keep]))
    assert list(got) == ["k", "s"]
    assert np.array_equal(got["k"], uk[keep][order])
    assert np.array_equal(got["s"], sums[keep][order])


def test_sql_in_lists(ex):
    rng = np.random.default_rng(5)
    n = 900_001
    k = rng.integers(-20, 20, n).astype(np.int64)
    f = (rng.integers(0, 8, n) / 4.0).astype(np.float64)
    v = rng.integers(0, 1 << 20, n) / 64.0
    t = {"k": dev(k, ex), "f": dev(f, ex), "v": dev(v, ex)}
    got = ex.sql("select k, sum(v), count(*) from t where k in (-3, 0, 7, 2.5, 99999999999999999999) "
                 "and f not in (0.25, 1.5) group by k", t)
    m = np.isin(k, [-3, 0, 7]) & ~np.isin(f, [0.25, 1.5])
    uk = np.unique(k[m])
    assert got["k"].tolist() == uk.tolist()
    assert got["count(*)"].tolist() == [int((k[m] == x).sum()) for x in uk]
    assert got["sum(v)"].tolist() == [float(v[m][k[m] == x].sum()) for x in uk]
    # an IN list nothing in the column can equal
    assert ex.sql("select count(*) from t where k in (0.5, 1.5)", t)["count(*)"].tolist() == [0]
    assert ex.sql("select count(*) from t where k not in (0.5)", t)["count(*)"].tolist() == [n]
    # the AggQuery path
    from nutdb_amd import Agg, AggQuery
    g = ex.groupby(AggQuery(keys=[t["k"]], aggs=[Agg("count")], preds=[(t["k"], "in", [1, 2, 3])]))
    keys, words = g.to_host_words()
    assert keys[:, 0].tolist() == [1, 2, 3] and words[:, 0].tolist() == [int((k == x).sum()) for x in (1, 2, 3)]


def test_sql_host_resident_columns(ex):
    """nut_column tagged NUT_COL_HOST (numpy arrays here): the library copies them into HBM
    for the call; results equal the device-resident run, for a group-by, an ORDER BY scan
    and a JOIN with one host and one device table."""
    rng = np.random.default_rng(81)
    n = 1_000_003
    k = rng.integers(0, 100, n).astype(np.int64)
    v = rng.integers(-1000, 1000, n).astype(np.float64) / 8.0
    w = rng.integers(0, 1 << 40, n).astype(np.int64)
    host = {"k": k, "v": v, "w": w}
    devc = {name: torch.from_numpy(a).to(ex.device) for name, a in host.items()}
    for sql in ("select k, sum(v) as s, count(*) as c, max(w) as m from t where w > 1000 group by k order by k",
                "select w, v from t where k < 3 order by v desc, w limit 1000",
                "select sum(v * 2) as s from t where k % 7 = 1 or w < 12345"):
        a, b = ex.sql(sql, host), ex.sql(sql, devc)
        for c in b:
            assert a[c].tolist() == b[c].tolist(), (sql, c)
    dim = {"dk": np.arange(100, dtype=np.int64), "dv": np.arange(100, dtype=np.int64) * 3}
    sql = "select dv, count(*) as c from t join dim on k = dk where w > 5000 group by dv order by dv"
    a = ex.sql(sql, host, right={n_: torch.from_numpy(x).to(ex.device) for n_, x in dim.items()})
    b = ex.sql(sql, devc, right=dim)
    m = w > 5000
    assert a["c"].tolist() == b["c"].tolist() == np.bincount(k[m], minlength=100).tolist()


def test_sql_scalar_subqueries(ex):
    """Uncorrelated scalar subqueries, executed first over the same columns (fixture 9's
    `c_acctbal > (select avg(c_acctbal) ...)`, fixture 4's HAVING > (select sum(..) * k),
    fixture 6's `= (select max(..))`), vs numpy on the same data.  Dyadic values: every
    sum and the avg division are exact / identically rounded, so comparisons are exact."""
    rng = np.random.default_rng(91)
    n = 1_000_003
    bal = (rng.integers(-2**20, 2**20, n) / 64.0).astype(np.float64)
    key = rng.integers(0, 100, n).astype(np.int64)
    qty = rng.integers(1, 50, n).astype(np.int64)
    cols = {"c_custkey": dev(np.arange(n, dtype=np.int64), ex), "c_acctbal": dev(bal, ex), "k": dev(key, ex),
            "qty": dev(qty, ex)}
    # WHERE col > (avg over a filtered set): a float placeholder
    pos = bal[bal > 0.0]
    avg = pos.sum() / len(pos)
    got = ex.sql("select c_custkey, c_acctbal from customer where c_acctbal > "
                 "(select avg(c_acctbal) from customer where c_acctbal > 0.00) and k < 50", cols)
    m = (bal > avg) & (key < 50)
    assert np.array_equal(got["c_custkey"], np.nonzero(m)[0]) and np.array_equal(got["c_acctbal"], bal[m])
    # = (select max(..)) over an int column, a count over the rows that equal it
    got = ex.sql("select count(*) as c from customer where qty = (select max(qty) from customer)", cols)
    assert int(got["c"][0]) == int((qty == qty.max()).sum())
    # two subqueries, one inside an expression (expression mode)
    got = ex.sql("select count(*) as c from customer where qty + 1 > (select max(qty) from customer) - 3 "
                 "and k >= (select min(k) from customer where qty > 40)", cols)
    kmin = key[qty > 40].min()
    assert int(got["c"][0]) == int(((qty + 1 > qty.max() - 3) & (key >= kmin)).sum())
    # HAVING sum(..) > (select sum(..) * 0.011 ...) over groups
    got = ex.sql("select k, sum(qty) as s from customer where qty > 2 group by k "
                 "having sum(qty) > (select sum(qty) * 0.011 from customer where qty > 2) order by k", cols,
                 group_hint=100)
    sel = qty > 2
    sums = np.bincount(key[sel], weights=qty[sel], minlength=100).astype(np.int64)
    bound = float(qty[sel].sum()) * 0.011
    want_k = np.nonzero(sums > bound)[0]
    assert np.array_equal(got["k"], want_k) and np.array_equal(got["s"], sums[want_k])
    # a global aggregate over no rows is one row of defaults (max 0), avg NaN acts as NULL
    got = ex.sql("select count(*) as c from customer where qty > (select max(qty) from customer where qty > 1000)",
                 cols)
    assert int(got["c"][0]) == n
    got = ex.sql("select count(*) as c from customer where c_acctbal > "
                 "(select avg(c_acctbal) from customer where qty > 1000)", cols)
    assert int(got["c"][0]) == 0
