"""GPU: GROUP BY beyond two key columns — computed keys, 3 / 5 / 8 keys
packed into the kernels' two key words, countUnique, and arithmetic over aggregates —
checked against the numpy expression oracle (oracle/expr.py: any number of keys, the
tuple ranked by numpy's lexicographic unique) and plain numpy.

  * key programs through the C ABI (nut_agg_spec.key_prog) vs groupby_prog, bit-exact;
  * SQL GROUP BY of 3, 5 and 8 keys of mixed ranges (small, 40-bit, full 64-bit raw words),
    their packing limits (a tuple needing more than 2 x 63 bits is refused, not truncated);
  * date parts (toYear / getYear ... toDayOfYear) as keys vs Python's calendar;
  * the reference fixture tests/sql/3.sql shape over one flat typed table: two String
    keys and getYear(l_shipdate) as the third, its WHERE and ORDER BY;
  * countUnique (fixture 7's aggregate) with 0-3 keys, masked arguments, a String
    argument, next to ordinary aggregates; arithmetic over aggregates in SELECT / HAVING /
    ORDER BY (TPC-H Q14's 100 * sum(..) / sum(..) shape).
Integer results bit-exact; f64 sums of non-dyadic values <= F64_SUM_RTOL relative.
"""
import datetime

import numpy as np
import pytest
import torch

from helpers import F64_SUM_RTOL, rel_err
from nutdb_amd import NutError, ProgQuery
from nutdb_amd.table import Table
from oracle.expr import date_part, groupby_prog

pytestmark = pytest.mark.gpu


def dev(x, ex):
    return torch.from_numpy(np.ascontiguousarray(x)).to(ex.device)


def oracle_groups(keys, aggs_cols, mask=None):
    """numpy: sorted distinct key tuples, and per group (count, sum / min / max of each
    aggs_cols array) — int64 arithmetic"""
    tup = np.stack(keys, axis=1)
    if mask is not None:
        tup = tup[mask]
        aggs_cols = [a[mask] for a in aggs_cols]
    uniq, inv = np.unique(tup, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    cnt = np.bincount(inv, minlength=len(uniq))
    out = [cnt]
    for a in aggs_cols:
        s = np.zeros(len(uniq), dtype=np.int64)
        np.add.at(s, inv, a)
        mn = np.full(len(uniq), np.iinfo(np.int64).max)
        np.minimum.at(mn, inv, a)
        mx = np.full(len(uniq), np.iinfo(np.int64).min)
        np.maximum.at(mx, inv, a)
        out += [s, mn, mx]
    return uniq, out


# ------------------------------------------------------------------ C ABI key programs
@pytest.mark.parametrize("seed", range(4))
def test_key_programs_abi(ex, seed):
    rng = np.random.default_rng(300 + seed)
    n = 300_001 + seed
    a = rng.integers(-5000, 5000, n).astype(np.int64)
    b = rng.integers(0, 2**40, n).astype(np.int64)
    d = rng.integers(-30000, 30000, n).astype(np.int64)  # days: years 1888 .. 2052
    v = rng.integers(-10**6, 10**6, n).astype(np.int64)
    cols = [a, b, d, v]
    k0 = [("col", 2), ("datepart", 0)]                                   # year
    k1 = [("col", 0), ("i64", 0, 7), ("mod",), ("col", 1), ("i64", 0, 20), ("shr",), ("bitxor",)]
    keys = [[k0], [k0, k1], [k1, [("col", 3), ("i64", 0, 0), ("gt",)]], [[("col", 2), ("datepart", 4)], k0]][seed]
    where = [("col", 0), ("i64", 0, 4000), ("lt",)] if seed % 2 else None
    aggs = [("sum", [("col", 3)], None), ("count", None, None), ("min", [("col", 1)], None),
            ("max", [("col", 3)], [("col", 0), ("i64", 0, 0), ("ge",)])]
    q = ProgQuery(keys=keys, cols=[dev(c, ex) for c in cols], where=where, aggs=aggs)
    gk, gw = ex.groupby(q, group_hint=[200, 4000, 30000, 1500][seed]).to_host_words()
    ok, ow, _ = groupby_prog(keys, cols, where, [({"sum": 0, "count": 1, "min": 2, "max": 3}[o], val, m)
                                                 for o, val, m in aggs])
    assert np.array_equal(gk, ok) and np.array_equal(gw, ow)


def test_key_program_division_by_zero(ex):
    n = 50_000
    a = np.arange(n, dtype=np.int64)
    z = (np.arange(n, dtype=np.int64) % 5)
    key = [("col", 0), ("col", 1), ("intdiv",)]
    with pytest.raises(NutError, match="division by zero"):
        ex.groupby(ProgQuery(keys=[key], cols=[dev(a, ex), dev(z, ex)], aggs=[("count", None, None)]))
    # rows failing WHERE never raise
    where = [("col", 1), ("i64", 0, 0), ("ne",)]
    q = ProgQuery(keys=[key], cols=[dev(a, ex), dev(z, ex)], where=where, aggs=[("count", None, None)])
    gk, gw = ex.groupby(q).to_host_words()
    ok, ow, _ = groupby_prog([key], [a, z], where, [(1, None, None)])
    assert np.array_equal(gk, ok) and np.array_equal(gw, ow)


# ------------------------------------------------------------------ SQL: N keys
def many_key_table(rng, n, nk):
    ranges = [(0, 3), (-2**39, 2**39), (0, 12), (-100, 100), (0, 2), (0, 70000), (0, 5), (-1, 1)]
    keys = [rng.integers(lo, hi + 1, n).astype(np.int64) for lo, hi in ranges[:nk]]
    # few distinct values of the wide key so that tuples repeat
    keys[1] = rng.choice(rng.integers(-2**39, 2**39, 64), n).astype(np.int64)
    return keys


@pytest.mark.parametrize("nk", [3, 5, 8])
def test_sql_group_by_n_keys(ex, nk):
    rng = np.random.default_rng(nk)
    n = 2_000_003
    keys = many_key_table(rng, n, nk)
    v = rng.integers(-10**9, 10**9, n).astype(np.int64)
    w = rng.integers(0, 1000, n).astype(np.int64)
    names = [f"k{j}" for j in range(nk)]
    cols = {nm: dev(k, ex) for nm, k in zip(names, keys)}
    cols.update(v=dev(v, ex), w=dev(w, ex))
    kl = ", ".join(names)
    got = ex.sql(f"select {kl}, count(*) as c, sum(v) as s, min(v) as mn, max(w) as mx from t "
                 f"where w < 900 group by {kl} order by {kl}", cols, group_hint=50_000)
    m = w < 900
    uniq, (cnt, s, mn, _, _, _, wmx) = oracle_groups(keys, [v, w], m)
    for j, nm in enumerate(names):
        assert np.array_equal(got[nm], uniq[:, j]), nm
    assert np.array_equal(got["c"], cnt) and np.array_equal(got["s"], s)
    assert np.array_equal(got["mn"], mn) and np.array_equal(got["mx"], wmx)
    # the same keys in another order group the same rows (key order = result order)
    rev = ", ".join(reversed(names))
    got2 = ex.sql(f"select {rev}, count(*) as c from t where w < 900 group by {rev}", cols)
    uniq2, (cnt2,) = oracle_groups(list(reversed(keys)), [], m)
    assert np.array_equal(np.stack([got2[nm] for nm in reversed(names)], axis=1), uniq2)
    assert np.array_equal(got2["c"], cnt2)


def test_sql_group_by_wide_keys(ex):
    """full-range int64 keys take raw words: two fit (and order as signed int64), a third
    full-range key is refused rather than truncated"""
    rng = np.random.default_rng(9)
    n = 500_000
    pool = rng.integers(-2**63, 2**63 - 1, 50, dtype=np.int64)
    a, b = rng.choice(pool, n), rng.choice(pool, n)
    c = rng.integers(0, 4, n).astype(np.int64)
    cols = {"a": dev(a, ex), "b": dev(b, ex), "c": dev(c, ex)}
    got = ex.sql("select a, b, count() as n from t group by a, b", cols)
    uniq, (cnt,) = oracle_groups([a, b], [])
    assert np.array_equal(got["a"], uniq[:, 0]) and np.array_equal(got["b"], uniq[:, 1])
    assert np.array_equal(got["n"], cnt)
    # a, c, b: word 0 = a (raw), word 1 = c | b does not fit 63 bits -> refused
    with pytest.raises(NutError, match="2 x 63 bits"):
        ex.sql("select a, c, b, count() from t group by a, c, b", cols)
    # a (raw word 0), then c and b % 1000 packed into word 1
    got = ex.sql("select a, c, b % 1000 as r, count() as n from t group by a, c, r", cols)
    uniq, (cnt,) = oracle_groups([a, c, np.fmod(b, 1000)], [])
    assert np.array_equal(np.stack([got["a"], got["c"], got["r"]], axis=1), uniq)
    assert np.array_equal(got["n"], cnt)


def test_sql_date_part_keys(ex):
    """seven keys: a day number and its six date parts (packing + DATEPART in one kernel)"""
    rng = np.random.default_rng(21)
    n = 1_000_000
    epoch = datetime.date(1970, 1, 1).toordinal()
    d = rng.integers(datetime.date(1, 1, 1).toordinal() - epoch, datetime.date(9999, 12, 31).toordinal() - epoch,
                     5000).astype(np.int64)
    d = rng.choice(d, n)
    got = ex.sql("select d, toYear(d) as y, getMonth(d) as m, toDayOfMonth(d) as dd, toQuarter(d) as q, "
                 "toDayOfWeek(d) as wd, getDayOfYear(d) as yd, count() as c from t "
                 "group by d, y, m, dd, q, wd, yd", {"d": dev(d, ex)}, group_hint=5000)
    days = np.unique(d)
    assert np.array_equal(got["d"], days)
    dates = [datetime.date.fromordinal(int(x) + epoch) for x in days]
    assert got["y"].tolist() == [x.year for x in dates]
    assert got["m"].tolist() == [x.month for x in dates]
    assert got["dd"].tolist() == [x.day for x in dates]
    assert got["q"].tolist() == [(x.month - 1) // 3 + 1 for x in dates]
    assert got["wd"].tolist() == [x.isoweekday() for x in dates]
    assert got["yd"].tolist() == [x.timetuple().tm_yday for x in dates]
    assert got["c"].tolist() == np.bincount(np.searchsorted(days, d)).tolist()
    # the clamp of impossible day numbers matches the oracle
    big = np.array([2**62, -2**62, 2**40 + 5, -(2**41), 0], dtype=np.int64)
    q = ProgQuery(keys=[[("col", 0), ("datepart", p)] for p in (0, 5)], cols=[dev(big, ex)],
                  aggs=[("count", None, None)])
    gk, _ = ex.groupby(q).to_host_words()
    want = np.unique(np.stack([date_part(big, 0), date_part(big, 5)], axis=1), axis=0)
    assert np.array_equal(gk, want)


def test_fixture3_shape(ex):
    """/root/reference/tests/sql/3.sql (TPC-H Q7) over one flat table: its subquery's
    columns as a typed table (nation names as String), getYear(l_shipdate) as the third
    GROUP BY key, the OR of nation pairs, BETWEEN toDate(..), ORDER BY all three keys."""
    rng = np.random.default_rng(33)
    n = 600_011
    nations = np.array(["FRANCE", "GERMANY", "BRAZIL", "CHINA", "PERU"], dtype=object)
    sn = nations[rng.integers(0, 5, n)]
    cn = nations[rng.integers(0, 5, n)]
    ship = rng.integers(datetime.date(1994, 6, 1).toordinal(), datetime.date(1997, 6, 1).toordinal(), n) \
        - datetime.date(1970, 1, 1).toordinal()
    price = rng.integers(90000, 10494900, n) / 128.0
    disc = rng.integers(0, 11, n) / 100.0
    t = Table(ex, """CREATE TABLE shipping (supp_nation String, cust_nation Dictionary(String), l_shipdate Date,
        l_extendedprice Float64, l_discount Float64)""")
    t.append(supp_nation=sn, cust_nation=cn, l_shipdate=ship, l_extendedprice=price, l_discount=disc)
    got = t.sql("""select supp_nation, cust_nation, getYear(l_shipdate) as l_year,
            sum(l_extendedprice * (1 - l_discount)) as revenue
        from shipping
        where ((supp_nation = 'FRANCE' and cust_nation = 'GERMANY')
            or (supp_nation = 'GERMANY' and cust_nation = 'FRANCE'))
          and l_shipdate between toDate('1995-01-01') and toDate('1996-12-31')
        group by supp_nation, cust_nation, l_year
        order by supp_nation, cust_nation, l_year""")
    lo = datetime.date(1995, 1, 1).toordinal() - datetime.date(1970, 1, 1).toordinal()
    hi = datetime.date(1996, 12, 31).toordinal() - datetime.date(1970, 1, 1).toordinal()
    m = (((sn == "FRANCE") & (cn == "GERMANY")) | ((sn == "GERMANY") & (cn == "FRANCE"))) & (ship >= lo) & (ship <= hi)
    year = date_part(ship, 0)
    rows = sorted({(a, b, int(y)) for a, b, y in zip(sn[m], cn[m], year[m])})
    assert list(zip(got["supp_nation"], got["cust_nation"], got["l_year"].tolist())) == rows
    assert len(rows) == 4
    for i, (a, b, y) in enumerate(rows):
        sel = m & (sn == a) & (cn == b) & (year == y)
        want = np.sum(price[sel] * (1 - disc[sel]))
        assert rel_err(np.array([got["revenue"][i]]), np.array([want])) <= F64_SUM_RTOL


# ------------------------------------------------------------------ countUnique
@pytest.mark.parametrize("nk", [0, 1, 2, 3])
def test_sql_count_unique(ex, nk):
    rng = np.random.default_rng(70 + nk)
    n = 1_500_007
    keys = [rng.integers(0, hi, n).astype(np.int64) for hi in (40, 7, 3)[:nk]]
    x = rng.integers(0, 5000, n).astype(np.int64)
    v = rng.integers(-100, 100, n).astype(np.int64)
    names = [f"k{j}" for j in range(nk)]
    cols = {nm: dev(k, ex) for nm, k in zip(names, keys)}
    cols.update(x=dev(x, ex), v=dev(v, ex))
    kl = ", ".join(names)
    sel = (kl + ", ") if nk else ""
    grp = f" group by {kl} order by {kl}" if nk else ""
    got = ex.sql(f"select {sel}countUnique(x) as u, uniqExact(case when v > 0 then x end) as up, sum(v) as s, "
                 f"count() as c from t where v != 7{grp}", cols, group_hint=1000)
    m = v != 7
    tup = np.stack(keys + [np.zeros(n, dtype=np.int64)], axis=1)[m]
    uniq, inv = np.unique(tup, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    xs, vs = x[m], v[m]
    u = [len(np.unique(xs[inv == g])) for g in range(len(uniq))]
    up = [len(np.unique(xs[(inv == g) & (vs > 0)])) for g in range(len(uniq))]
    s = [int(vs[inv == g].sum()) for g in range(len(uniq))]
    for j, nm in enumerate(names):
        assert np.array_equal(got[nm], uniq[:, j])
    assert got["u"].tolist() == u and got["up"].tolist() == up
    assert got["s"].tolist() == s and got["c"].tolist() == np.bincount(inv).tolist()


def test_fixture7_shape(ex):
    """/root/reference/tests/sql/7.sql (TPC-H Q16) without its subquery: countUnique of
    the supplier per (brand, type, size) — three keys, two of them String — NOT LIKE, a
    long IN list, a NOT IN list standing in for the subquery, ORDER BY the count desc."""
    rng = np.random.default_rng(77)
    n = 800_003
    brands = np.array([f"Brand#{i}{j}" for i in range(1, 6) for j in range(1, 6)], dtype=object)
    types = np.array(["MEDIUM POLISHED TIN", "SMALL PLATED STEEL", "LARGE BRUSHED BRASS", "ECONOMY ANODIZED NICKEL",
                      "MEDIUM POLISHED COPPER", "STANDARD BURNISHED TIN"], dtype=object)
    pb, pt = brands[rng.integers(0, len(brands), n)], types[rng.integers(0, len(types), n)]
    size = rng.integers(1, 51, n)
    supp = rng.integers(0, 2000, n)
    pk = rng.integers(0, 100, n)
    psk = np.where(rng.random(n) < 0.8, pk, rng.integers(0, 100, n))
    t = Table(ex, """CREATE TABLE partsupp (p_partkey Int64, ps_partkey Int64, p_brand Dictionary(String),
        p_type String, p_size Int32, ps_suppkey Int64)""")
    t.append(p_partkey=pk, ps_partkey=psk, p_brand=pb, p_type=pt, p_size=size.astype(np.int32), ps_suppkey=supp)
    bad = [3, 77, 1000, 1999]
    got = t.sql(f"""select p_brand, p_type, p_size, countUnique(ps_suppkey) as supplier_cnt
        from partsupp
        where p_partkey = ps_partkey and p_brand <> 'Brand#45' and p_type not like 'MEDIUM POLISHED%'
          and p_size in (49, 14, 23, 45, 19, 3, 36, 9) and ps_suppkey not in ({", ".join(map(str, bad))})
        group by p_brand, p_type, p_size
        order by supplier_cnt desc, p_brand, p_type, p_size""")
    m = (pk == psk) & (pb != "Brand#45") & ~np.array([s.startswith("MEDIUM POLISHED") for s in pt]) \
        & np.isin(size, [49, 14, 23, 45, 19, 3, 36, 9]) & ~np.isin(supp, bad)
    groups = {}
    for b, ty, sz, sp in zip(pb[m], pt[m], size[m], supp[m]):
        groups.setdefault((b, ty, int(sz)), set()).add(int(sp))
    want = sorted(((-len(s), k) for k, s in groups.items()))
    assert list(zip(got["p_brand"], got["p_type"], got["p_size"].tolist())) == [k for _, k in want]
    assert got["supplier_cnt"].tolist() == [-c for c, _ in want]


def test_count_unique_of_strings_and_limits(ex):
    rng = np.random.default_rng(5)
    n = 200_000
    words = np.array([f"w{i}" for i in range(300)], dtype=object)
    s = words[rng.integers(0, 300, n)]
    k = rng.integers(0, 4, n)
    t = Table(ex, "CREATE TABLE t (k Int64, s String)")
    t.append(k=k, s=s)
    got = t.sql("select k, countUnique(s) as u from t group by k order by k")
    assert got["u"].tolist() == [len(set(s[k == g])) for g in range(4)]
    with pytest.raises(NutError, match="float64"):
        ex.sql("select countUnique(f) from t", {"f": dev(rng.random(10), ex)})


# ------------------------------------------------------------------ arithmetic over aggregates
def test_sql_aggregate_arithmetic(ex):
    rng = np.random.default_rng(14)
    n = 1_000_003
    k = rng.integers(0, 9, n).astype(np.int64)
    a = rng.integers(0, 1000, n).astype(np.int64)
    p = rng.integers(90000, 10494900, n) / 128.0
    promo = rng.integers(0, 2, n).astype(np.int64)
    cols = {"k": dev(k, ex), "a": dev(a, ex), "p": dev(p, ex), "promo": dev(promo, ex)}
    got = ex.sql("""select k, sum(a) / count() as mean, sum(a) - min(a) * 2 as d, intDiv(sum(a), 7) % 5 as r,
            100.00 * sum(case when promo = 1 then p else 0 end) / sum(p) as promo_revenue,
            k * 10 + 1 as k10, 0 - sum(a) as neg
        from t group by k having sum(a) / count() > 499 or k = 3 order by promo_revenue desc, k""", cols)
    rows = []
    for g in range(9):
        sel = k == g
        sa, cnt, mn = int(a[sel].sum()), int(sel.sum()), int(a[sel].min())
        pr = 100.0 * p[sel & (promo == 1)].sum() / p[sel].sum()
        if sa / cnt > 499 or g == 3:
            rows.append((g, sa / cnt, sa - mn * 2, (sa // 7) % 5, pr, g * 10 + 1, -sa))
    rows.sort(key=lambda r: (-r[4], r[0]))
    assert got["k"].tolist() == [r[0] for r in rows]
    assert got["d"].tolist() == [r[2] for r in rows] and got["r"].tolist() == [r[3] for r in rows]
    assert got["k10"].tolist() == [r[5] for r in rows] and got["neg"].tolist() == [r[6] for r in rows]
    assert got["mean"].dtype == np.float64 and np.allclose(got["mean"], [r[1] for r in rows], rtol=1e-15)
    assert rel_err(got["promo_revenue"], np.array([r[4] for r in rows])) <= 4 * F64_SUM_RTOL
    with pytest.raises(NutError, match="division by zero"):
        ex.sql("select k, sum(a) % (count() - count()) from t group by k", cols)
