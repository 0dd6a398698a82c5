"""GPU parity of the hash join (csrc/join.hip) and the gather that carries columns through
a join index, against the numpy oracle (oracle/oracle.py join_i64).  Pairs come out in
probe-row order; the build rows of one probe row are in unspecified order, so each probe
row's build rows are compared sorted."""
import numpy as np
import pytest
import torch

from test_gpu_exec import I64_MAX, I64_MIN, dev, host

pytestmark = pytest.mark.gpu

HOW = ["inner", "left", "semi", "anti"]


def canon(pi, bi):
    o = np.lexsort((bi, pi))
    return pi[o], bi[o]


def check(ex, orc, b, p, how, passes=1, any_order=False):
    pi, bi = ex.join_i64(dev(b, ex), dev(p, ex), how, passes=passes, any_order=any_order)
    pi, bi = host(pi), host(bi)
    wp, wb = orc.join_i64(b, p, how)
    if not any_order:
        assert np.all(pi[1:] >= pi[:-1]), "pairs not in probe-row order"
    gp, gb = canon(pi, bi)
    assert np.array_equal(gp, wp) and np.array_equal(gb, wb), how


@pytest.mark.parametrize("how", HOW)
@pytest.mark.parametrize("nb,np_", [(0, 1000), (1000, 0), (1, 1), (100, 5000), (4096, 4097), (100_000, 1_000_003)])
def test_join_unique_build(ex, orc, how, nb, np_):
    rng = np.random.default_rng(nb + np_)
    b = rng.permutation(np.arange(nb, dtype=np.int64) * 7 - 1000)
    p = rng.integers(-2000, 7 * max(nb, 1), np_).astype(np.int64)
    check(ex, orc, b, p, how)


@pytest.mark.parametrize("passes", [1, 2])
@pytest.mark.parametrize("how", HOW)
def test_join_duplicates_both_sides(ex, orc, how, passes):
    """Repeated build keys: INNER / LEFT produce more pairs than probe rows, so the
    one-pass form hits NUT_ERR_CAPACITY and runs again at the exact size."""
    rng = np.random.default_rng(5)
    b = rng.integers(0, 300, 20_000).astype(np.int64)
    p = rng.integers(-50, 350, 30_001).astype(np.int64)
    check(ex, orc, b, p, how, passes)


@pytest.mark.parametrize("how", HOW)
def test_join_two_pass_api(ex, orc, how):
    rng = np.random.default_rng(15)
    b = rng.permutation(np.arange(70_000, dtype=np.int64) * 5)
    p = rng.integers(-100, 400_000, 1_000_003).astype(np.int64)
    check(ex, orc, b, p, how, passes=2)


@pytest.mark.parametrize("how", HOW)
def test_join_region_build(ex, orc, how):
    """> 2^20 build rows: the table is built region by region in LDS (hash_partition16 +
    hj_region_build_kernel), with repeated keys (duplicate check inside the regions)."""
    rng = np.random.default_rng(31)
    b = rng.integers(0, 1_500_000, 2_100_000).astype(np.int64)
    p = rng.integers(-100_000, 1_600_000, 3_000_001).astype(np.int64)
    check(ex, orc, b, p, how)


def test_join_region_overflow_falls_back(ex, orc):
    """1.2e6 copies of one key cannot fit a 8192-slot region: the global CAS build runs."""
    b = np.concatenate([np.full(1_200_000, 42, dtype=np.int64), np.arange(1_000_000, dtype=np.int64) * 5 + 7])
    p = np.array([42, 7, 8, 42, 12, -1], dtype=np.int64)
    check(ex, orc, b, p, "inner")
    check(ex, orc, b, p, "semi")


def test_join_long_runs(ex, orc):
    """Clustered hashes: 1000 copies of each of 3 keys build long probe runs; tiles mix
    rows with thousands of matches and rows with none."""
    rng = np.random.default_rng(21)
    b = np.repeat(np.array([7, -7, 2**40], dtype=np.int64), 1000)
    p = rng.choice(np.array([7, -7, 2**40, 8, 9], dtype=np.int64), 5_000)
    check(ex, orc, b, p, "inner")
    check(ex, orc, b, p, "left")
    check(ex, orc, b, p, "anti")


@pytest.mark.parametrize("how", HOW)
def test_join_extreme_keys(ex, orc, how):
    rng = np.random.default_rng(9)
    pool = np.array([I64_MIN, I64_MAX, 0, -1, 1, 123456789012345], dtype=np.int64)
    b = pool[rng.integers(0, 4, 50)]
    p = pool[rng.integers(0, len(pool), 10_000)]
    check(ex, orc, b, p, how)


@pytest.mark.parametrize("passes", [1, 2])
@pytest.mark.parametrize("how", HOW)
def test_join_any_order(ex, orc, how, passes):
    """NUT_JOIN_ANY_ORDER (the unordered probe, used under aggregates): the same pair
    multiset as the ordered join — unique keys, repeated keys past the first capacity,
    region-built tables, long runs, extreme keys, empty sides."""
    rng = np.random.default_rng(77)
    cases = [
        (rng.permutation(np.arange(100_000, dtype=np.int64) * 7 - 1000), rng.integers(-2000, 700_000, 1_000_003)),
        (rng.integers(0, 300, 20_000), rng.integers(-50, 350, 30_001)),
        (rng.integers(0, 1_500_000, 2_100_000), rng.integers(-100_000, 1_600_000, 3_000_001)),
        (np.repeat(np.array([7, -7, 2**40], dtype=np.int64), 1000), rng.choice(np.array([7, -7, 2**40, 8, 9]), 5_000)),
        (np.array([I64_MIN, I64_MAX, 0, -1], dtype=np.int64)[rng.integers(0, 4, 50)],
         np.array([I64_MIN, I64_MAX, 0, -1, 1, 5], dtype=np.int64)[rng.integers(0, 6, 10_000)]),
        (np.zeros(0, np.int64), rng.integers(0, 9, 1000)),
        (rng.integers(0, 9, 1000), np.zeros(0, np.int64)),
        (np.array([3], np.int64), np.array([3], np.int64)),
    ]
    for b, p in cases:
        check(ex, orc, b.astype(np.int64), p.astype(np.int64), how, passes=passes, any_order=True)


@pytest.mark.parametrize("match", [1, 0])
@pytest.mark.parametrize("how", HOW)
def test_join_ordered_one_vs_two_pass(ex, orc, opts, how, match):
    """The ordered write with NUT_OPT_JOIN_MATCH on (default: walks into a match array, then
    the ordered write-out from it, whenever no probe row can match two build rows) and off
    (one ordered pass): unique keys (two passes), repeated keys (INNER / LEFT stay one pass;
    SEMI / ANTI take two), a region-built table, extreme keys, tile-boundary sizes."""
    opts(join_match=match)
    rng = np.random.default_rng(88)
    cases = [
        (rng.permutation(np.arange(100_000, dtype=np.int64) * 7 - 1000), rng.integers(-2000, 700_000, 1_000_003)),
        (rng.integers(0, 300, 20_000), rng.integers(-50, 350, 30_001)),
        (rng.permutation(np.arange(2_100_000, dtype=np.int64) * 3), rng.integers(-100_000, 6_400_000, 3_000_001)),
        (np.array([I64_MIN, I64_MAX, 0, -1], dtype=np.int64),
         np.array([I64_MIN, I64_MAX, 0, -1, 1, 5], dtype=np.int64)[rng.integers(0, 6, 10_000)]),
        (np.array([3], np.int64), np.array([3], np.int64)),
        (rng.permutation(np.arange(5000, dtype=np.int64)), rng.integers(0, 10_000, 4096)),
        (rng.permutation(np.arange(5000, dtype=np.int64)), rng.integers(0, 10_000, 4097)),
    ]
    for b, p in cases:
        check(ex, orc, b.astype(np.int64), p.astype(np.int64), how)


def test_join_large_property(ex, orc):
    """1e7 unique build keys, 2e8 probe keys (~90 % matching): count and a checksum of the
    pairs against numpy."""
    nb, np_ = 10_000_000, 200_000_000
    b = ex.gen_column(0, 0x71, nb)  # unique with overwhelming probability (62-bit)
    bh = host(b)
    sel = ex.gen_column(0, 0x72, np_)  # probe: every 10th row misses
    idx = (sel % nb)
    p = torch.where(sel % 10 == 0, sel | (1 << 62), b[idx])
    pi, bi = ex.join_i64(b, p, "inner")
    hp = host(p)
    miss = (host(sel) % 10) == 0
    assert len(pi) == int((~miss).sum())
    assert np.array_equal(host(pi), np.nonzero(~miss)[0])
    assert np.array_equal(bh[host(bi)], hp[~miss])
    # the unordered probe: the same pairs once sorted by probe row
    ui, ub = ex.join_i64(b, p, "inner", any_order=True)
    o = torch.argsort(ui)
    assert torch.equal(ui[o], pi) and torch.equal(ub[o], bi)


def test_gather_null_and_f64(ex):
    col = torch.arange(10, dtype=torch.float64, device=ex.device) * 1.5
    idx = torch.tensor([3, -1, 0, 9, -1], dtype=torch.int64, device=ex.device)
    out = host(ex.gather(col, idx, null=-0.25))
    assert out.tolist() == [4.5, -0.25, 0.0, 13.5, -0.25]
    icol = torch.tensor([I64_MIN, 7, I64_MAX], dtype=torch.int64, device=ex.device)
    assert host(ex.gather(icol, torch.tensor([2, 0, -1], device=ex.device), null=-9)).tolist() == [I64_MAX, I64_MIN, -9]


# ------------------------------------------------------------------ SQL: JOIN plans
# (nut_plan_execute2: hash join on the ON columns, gathers, then the plan's group-by /
# scan on the joined rows).  Expected values: the numpy join oracle + pandas group-by.
# The reference parses JOINs but executes none: semantics are this build's (SQL's, with
# ClickHouse-style non-Nullable aggregate results), parity pinned by the numpy oracle.
import pandas as pd  # noqa: E402

from nutdb_amd import NutError  # noqa: E402


def tables(seed, norders, nlines, miss=0.2):
    rng = np.random.default_rng(seed)
    o_okey = rng.permutation(np.arange(norders, dtype=np.int64) * 3 + 11)
    o_cust = rng.integers(0, 50, norders).astype(np.int64)
    hit = o_okey[rng.integers(0, norders, nlines)] if norders else np.full(nlines, 5, dtype=np.int64)
    l_okey = np.where(rng.random(nlines) < miss, rng.integers(0, 3 * max(norders, 1), nlines) * 3 + 12, hit).astype(np.int64)
    l_qty = rng.integers(1, 60, nlines).astype(np.int64)
    l_price = rng.integers(-4096, 4096, nlines).astype(np.float64) / 32.0  # dyadic: sums exact
    return ({"o_okey": o_okey, "o_cust": o_cust}, {"l_okey": l_okey, "l_qty": l_qty, "l_price": l_price})


def joined(orc, left, lkey, right, rkey, how):
    """numpy join of left (preserved for outer / semi / anti) with right: a DataFrame with
    every column of both, NaN-free; `matched` marks rows with a right row."""
    pi, bi = orc.join_i64(right[rkey], left[lkey], how)
    d = {k: v[pi] for k, v in left.items()}
    if how in ("inner", "left"):
        for k, v in right.items():
            d[k] = np.where(bi >= 0, v[np.maximum(bi, 0)], 0).astype(v.dtype)
    d["matched"] = bi >= 0
    return pd.DataFrame(d)


def on_dev(ex, t):
    return {k: dev(v, ex) for k, v in t.items()}


@pytest.mark.parametrize("sizes", [(20_000, 100_000), (200_000, 50_000), (0, 1000), (1000, 0)])
def test_sql_inner_join_groupby(ex, orc, sizes):
    orders, lines = tables(1, *sizes)
    sql = """select o_cust, sum(l_qty) as q, count(*) as c, min(l_price) as mn, max(l_qty) as mx,
               sum(l_price) as p
             from lineitem join orders on l_okey = o_okey where l_qty > 3 group by o_cust order by o_cust"""
    got = ex.sql(sql, on_dev(ex, lines), right=on_dev(ex, orders))
    j = joined(orc, lines, "l_okey", orders, "o_okey", "inner")
    g = j[j.l_qty > 3].groupby("o_cust").agg(q=("l_qty", "sum"), c=("l_qty", "size"), mn=("l_price", "min"),
                                            mx=("l_qty", "max"), p=("l_price", "sum"))
    assert got["o_cust"].tolist() == g.index.tolist()
    for c in ("q", "c", "mn", "mx", "p"):
        assert got[c].tolist() == g[c].tolist(), c


@pytest.mark.parametrize("right", [False, True])
def test_sql_left_outer_join_groupby(ex, orc, right):
    orders, lines = tables(2, 30_000, 60_000, miss=0.3)
    orders["o_cust"][:40] = 1000  # customer 1000: orders with no line (below)
    lines["l_okey"][np.isin(lines["l_okey"], orders["o_okey"][:40])] = -5
    body = ("from orders left join lineitem on o_okey = l_okey" if not right
            else "from lineitem right outer join orders on l_okey = o_okey")
    sql = f"""select o_cust, count(*) as c, count(l_qty) as cl, sum(l_qty) as s, sum(l_price) as p,
                avg(l_qty) as a, max(case when l_qty > 50 then l_price end) as mx
              {body} where o_cust >= 10 group by o_cust order by o_cust"""
    got = ex.sql(sql, on_dev(ex, lines if right else orders), right=on_dev(ex, orders if right else lines))
    j = joined(orc, orders, "o_okey", lines, "l_okey", "left")
    j = j[j.o_cust >= 10]
    m = j[j.matched]
    g = j.groupby("o_cust").size()
    assert got["o_cust"].tolist() == g.index.tolist()
    assert got["c"].tolist() == g.tolist()
    cl = m.groupby("o_cust").size().reindex(g.index, fill_value=0)
    assert got["cl"].tolist() == cl.tolist()
    assert got["s"].tolist() == m.groupby("o_cust").l_qty.sum().reindex(g.index, fill_value=0).tolist()
    assert got["p"].tolist() == m.groupby("o_cust").l_price.sum().reindex(g.index, fill_value=0.0).tolist()
    i1000 = g.index.tolist().index(1000)
    assert got["cl"][i1000] == 0 and got["s"][i1000] == 0 and got["c"][i1000] == 40
    a = (m.groupby("o_cust").l_qty.sum() / m.groupby("o_cust").size()).reindex(g.index)
    keep = g.index != 1000
    assert np.array_equal(got["a"][keep], a[keep].to_numpy())
    big = m[m.l_qty > 50].groupby("o_cust").l_price.max()
    for i, cst in enumerate(g.index):
        if cst in big.index:
            assert got["mx"][i] == big[cst]


@pytest.mark.parametrize("how", ["semi", "anti"])
def test_sql_semi_anti_join(ex, orc, how):
    orders, lines = tables(3, 50_000, 80_000, miss=0.5)
    sql = f"""select o_cust, count(*) as c, sum(o_okey) as s from orders left {how} join lineitem
              on o_okey = l_okey group by o_cust order by o_cust"""
    got = ex.sql(sql, on_dev(ex, orders), right=on_dev(ex, lines))
    j = joined(orc, orders, "o_okey", lines, "l_okey", how)
    g = j.groupby("o_cust").agg(c=("o_okey", "size"), s=("o_okey", "sum"))
    assert got["o_cust"].tolist() == g.index.tolist()
    assert got["c"].tolist() == g.c.tolist() and got["s"].tolist() == g.s.tolist()
    # the RIGHT form preserves the JOIN source; SEMI may read the other ON column
    sql = f"select l_okey from lineitem right {how} join orders on l_okey = o_okey"
    if how == "semi":
        got = ex.sql(sql, on_dev(ex, lines), right=on_dev(ex, orders))
        assert got["l_okey"].tolist() == j.o_okey.tolist()
    else:
        with pytest.raises(NutError, match="preserved table"):
            ex.sql(sql, on_dev(ex, lines), right=on_dev(ex, orders))


@pytest.mark.parametrize("sizes", [(30_000, 60_000), (0, 1000), (1000, 0)])
def test_sql_full_outer_join(ex, orc, sizes):
    """FULL OUTER JOIN = the LEFT join's pairs + the JOIN source's unmatched rows; each
    side's aggregates skip the rows where that side is NULL (pandas outer merge)."""
    orders, lines = tables(6, *sizes, miss=0.3)
    if len(orders["o_okey"]):
        orders["o_cust"][:40] += 7
        lines["l_okey"][np.isin(lines["l_okey"], orders["o_okey"][:40])] = -5  # orders with no line
    sql = """select count(*) as c, count(l_qty) as cl, sum(l_qty) as s, count(o_cust) as co,
                    sum(o_cust) as so, sum(l_price) as p, min(o_okey) as mn, max(l_okey) as mx
             from orders full outer join lineitem on o_okey = l_okey"""
    got = ex.sql(sql, on_dev(ex, orders), right=on_dev(ex, lines))
    m = pd.DataFrame(orders).merge(pd.DataFrame(lines), left_on="o_okey", right_on="l_okey", how="outer")
    assert got["c"].tolist() == [len(m)]
    assert got["cl"].tolist() == [int(m.l_qty.notna().sum())]
    assert got["co"].tolist() == [int(m.o_cust.notna().sum())]
    assert got["s"].tolist() == [int(m.l_qty.sum())]
    assert got["so"].tolist() == [int(m.o_cust.sum())]
    assert got["p"].tolist() == [float(m.l_price.sum())]  # dyadic values: exact in any order
    if m.o_okey.notna().any():
        assert got["mn"].tolist() == [int(m.o_okey.min())]
    if m.l_okey.notna().any():
        assert got["mx"].tolist() == [int(m.l_okey.max())]
    with pytest.raises(NutError, match="FULL OUTER JOIN: column 'o_cust'"):
        ex.sql("select o_cust, count(*) from orders full join lineitem on o_okey = l_okey group by o_cust",
               on_dev(ex, orders), right=on_dev(ex, lines))


def test_sql_join_scan_and_sort(ex, orc):
    orders, lines = tables(4, 10_000, 40_000)
    got = ex.sql("select l_qty from lineitem join orders on l_okey = o_okey where l_qty >= 30",
                 on_dev(ex, lines), right=on_dev(ex, orders))
    j = joined(orc, lines, "l_okey", orders, "o_okey", "inner")
    assert got["l_qty"].tolist() == j.l_qty[j.l_qty >= 30].tolist()  # joined rows in probe-row order
    got = ex.sql("select o_okey from orders join lineitem on o_okey = l_okey order by o_okey desc limit 100",
                 on_dev(ex, orders), right=on_dev(ex, lines))
    assert got["o_okey"].tolist() == sorted(j.o_okey.tolist(), reverse=True)[:100]


def test_sql_join_errors(ex):
    orders, lines = tables(5, 200, 200)  # equal lengths: the binding checks pass, the plan errors
    o, l_ = on_dev(ex, orders), on_dev(ex, lines)
    with pytest.raises(NutError, match="may only appear inside aggregates"):
        ex.sql("select o_cust, count(*) from orders left join lineitem on o_okey = l_okey where l_qty > 3 "
               "group by o_cust", o, right=l_)
    with pytest.raises(NutError, match="may only appear inside aggregates"):
        ex.sql("select l_qty, count(*) from orders left join lineitem on o_okey = l_okey group by l_qty", o, right=l_)
    with pytest.raises(NutError, match="in both tables"):
        ex.sql("select o_cust, count(*) from orders join lineitem on o_okey = l_okey group by o_cust",
               o, right={**l_, "o_cust": o["o_cust"]})
    with pytest.raises(NutError, match="must be int64"):
        ex.sql("select count(*) from orders join lineitem on o_okey = l_price", o, right=l_)
    with pytest.raises(NutError, match="a column of each table"):
        ex.sql("select count(*) from orders join lineitem on o_okey = o_cust", o, right=l_)
    from nutdb_amd.sql import Plan
    with pytest.raises(NutError, match="nut_plan_execute2"):
        Plan("select count(*) from orders join lineitem on o_okey = l_okey").execute(ex, {**o, **l_})


def test_sql_inner_join_large(ex, orc):
    """1e6 orders x 8e6 lines: the TPC-H-shaped join + group-by (Q3/Q10 style)."""
    orders, lines = tables(6, 1_000_000, 8_000_000)
    sql = """select o_cust, count(*) as c, sum(l_qty) as q from lineitem join orders on l_okey = o_okey
             group by o_cust order by o_cust"""
    got = ex.sql(sql, on_dev(ex, lines), right=on_dev(ex, orders))
    j = joined(orc, lines, "l_okey", orders, "o_okey", "inner")
    g = j.groupby("o_cust").agg(c=("l_qty", "size"), q=("l_qty", "sum"))
    assert got["o_cust"].tolist() == g.index.tolist()
    assert got["c"].tolist() == g.c.tolist() and got["q"].tolist() == g.q.tolist()


def test_sql_join_qualified_same_name_keys(ex, orc):
    """`ON o.okey = l.okey`: both tables name their key `okey`; qualifiers (table names or
    AS aliases) pick the table, unqualified names must be unique across the two."""
    orders, lines = tables(7, 30_000, 90_000)
    o = {"okey": dev(orders["o_okey"], ex), "cust": dev(orders["o_cust"], ex)}
    li = {"okey": dev(lines["l_okey"], ex), "qty": dev(lines["l_qty"], ex)}
    j = joined(orc, lines, "l_okey", orders, "o_okey", "inner")
    g = j.groupby("o_cust").agg(c=("l_qty", "size"), q=("l_qty", "sum"))
    for sql in ["select cust, count(*) as c, sum(qty) as q from lineitem as l join orders as o "
                "on l.okey = o.okey group by cust order by cust",
                "select o.cust, count(*) as c, sum(lineitem.qty) as q from lineitem join orders as o "
                "on lineitem.okey = o.okey group by o.cust order by o.cust"]:
        got = ex.sql(sql, li, right=o)
        assert list(got.values())[0].tolist() == g.index.tolist()
        assert got["c"].tolist() == g.c.tolist() and got["q"].tolist() == g.q.tolist()
    with pytest.raises(NutError, match="names neither"):
        ex.sql("select count(*) from lineitem as l join orders as o on x.okey = o.okey", li, right=o)
    with pytest.raises(NutError, match="in both tables"):
        ex.sql("select count(*) from lineitem as l join orders as o on okey = o.okey", li, right=o)


def test_sql_join_pushdown_mixed_where(ex, orc):
    """WHERE conjuncts on one table are pushed below the join (nut_select_rows on that
    table); a conjunct reading both tables stays above it; OR across tables stays whole."""
    orders, lines = tables(8, 40_000, 150_000)
    j = joined(orc, lines, "l_okey", orders, "o_okey", "inner")
    cases = [
        ("l_qty > 3 and o_cust < 30 and l_qty > o_cust", (j.l_qty > 3) & (j.o_cust < 30) & (j.l_qty > j.o_cust)),
        ("(l_qty > 50 or o_cust = 7) and l_price >= 0", ((j.l_qty > 50) | (j.o_cust == 7)) & (j.l_price >= 0)),
        ("l_qty in (5, 6, 7) and o_cust != 3", j.l_qty.isin([5, 6, 7]) & (j.o_cust != 3)),
    ]
    for where, m in cases:
        got = ex.sql(f"select o_cust, count(*) as c, sum(l_qty) as q from lineitem join orders on l_okey = o_okey "
                     f"where {where} group by o_cust order by o_cust", on_dev(ex, lines), right=on_dev(ex, orders))
        g = j[m].groupby("o_cust").agg(c=("l_qty", "size"), q=("l_qty", "sum"))
        assert got["o_cust"].tolist() == g.index.tolist(), where
        assert got["c"].tolist() == g.c.tolist() and got["q"].tolist() == g.q.tolist(), where
    # a scan with a pushed-down predicate keeps probe-row order
    got = ex.sql("select l_qty from lineitem join orders on l_okey = o_okey where o_cust = 4 and l_qty < 20",
                 on_dev(ex, lines), right=on_dev(ex, orders))
    assert got["l_qty"].tolist() == j.l_qty[(j.o_cust == 4) & (j.l_qty < 20)].tolist()


def test_q12_join_bench_workload_parity(ex, orc):
    """bench.py's q12join workload (TPC-H Q12 as written, pushdown + join + expression
    group-by) on 2e6 lines against its own CPU baseline computation."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import bench
    from nutdb_amd.sql import Plan
    n = 2_000_000
    od, ld = bench.q12j_tables(lambda k, seed, m, a, b: ex.gen_column(k, seed, m, a=a, b=b), n)
    got = Plan(bench.Q12J_SQL).execute_join(ex, od, ld, group_hint=8)
    o, li = bench.q12j_tables(lambda k, seed, m, a, b: orc.gen_column(k, seed, m, a=a, b=b), n)
    m = (np.isin(li["l_shipmode"], [3, 5]) & (li["l_commitdate"] < li["l_receiptdate"])
         & (li["l_shipdate"] < li["l_commitdate"]))
    ids = np.nonzero(m)[0]
    pi, bi = orc.join_i64(o["o_orderkey"], li["l_orderkey"][ids], "inner")
    pr, mode = o["o_orderpriority"][bi], li["l_shipmode"][ids[pi]]
    hi = (pr == 1) | (pr == 2)
    assert got["l_shipmode"].tolist() == [3, 5]
    assert got["high_line_count"].tolist() == [int(np.sum(hi & (mode == s))) for s in (3, 5)]
    assert got["low_line_count"].tolist() == [int(np.sum(~hi & (mode == s))) for s in (3, 5)]


def test_sql_three_table_join(ex, orc):
    """lineitem JOIN orders JOIN customer (nut_plan_executen): pushed-down WHERE on two
    tables, a cross-table conjunct above the joins, group-by on the third table's column."""
    orders, lines = tables(9, 40_000, 160_000)
    rng = np.random.default_rng(90)
    ncust = 50
    cust = {"c_key": rng.permutation(ncust).astype(np.int64), "c_nation": rng.integers(0, 8, ncust).astype(np.int64)}
    j = joined(orc, lines, "l_okey", orders, "o_okey", "inner")
    cn = dict(zip(cust["c_key"].tolist(), cust["c_nation"].tolist()))
    j["c_nation"] = [cn[k] for k in j.o_cust.tolist()]
    m = (j.l_qty > 10) & (j.c_nation < 6) & (j.l_qty > j.o_cust)
    g = j[m].groupby("c_nation").agg(n=("l_qty", "size"), q=("l_qty", "sum"))
    got = ex.sql("select c_nation, count(*) as n, sum(l_qty) as q from lineitem join orders on l_okey = o_okey "
                 "join customer on o_cust = c_key where l_qty > 10 and c_nation < 6 and l_qty > o_cust "
                 "group by c_nation order by c_nation", on_dev(ex, lines), right=[on_dev(ex, orders), on_dev(ex, cust)])
    assert got["c_nation"].tolist() == g.index.tolist()
    assert got["n"].tolist() == g.n.tolist() and got["q"].tolist() == g.q.tolist()


def test_sql_join_using_and_multi_key(ex, orc):
    """JOIN ... USING (k) (the shared name binds to the preserved table) and joins on two
    key columns (USING (a, b) / ON a = b AND c = d: hash join on the first, the rest
    filtered above the join) against pandas merges."""
    rng = np.random.default_rng(71)
    n1, n2 = 3000, 40_000
    t1 = {"k": rng.permutation(n1).astype(np.int64), "s": rng.integers(0, 4, n1).astype(np.int64),
          "v1": rng.integers(0, 100, n1).astype(np.int64)}
    t2 = {"k": rng.integers(-100, n1 + 100, n2).astype(np.int64), "s": rng.integers(0, 4, n2).astype(np.int64),
          "v2": rng.integers(0, 100, n2).astype(np.int64)}
    d1, d2 = pd.DataFrame(t1), pd.DataFrame(t2)
    got = ex.sql("select k, count(*) as c, sum(v2) as s2 from t1 join t2 using (k) where k < 1000 "
                 "group by k order by k", on_dev(ex, t1), right=on_dev(ex, t2))
    m = d1.merge(d2, on="k")
    g = m[m.k < 1000].groupby("k").agg(c=("v2", "size"), s2=("v2", "sum"))
    assert got["k"].tolist() == g.index.tolist() and got["c"].tolist() == g.c.tolist()
    assert got["s2"].tolist() == g.s2.tolist()
    m2 = d1.merge(d2, on=["k", "s"])
    for sql in ("select s, count(*) as c, sum(v1) as a, sum(v2) as b from t1 join t2 using (k, s) group by s order by s",
                "select t1.s, count(*) as c, sum(v1) as a, sum(v2) as b from t1 join t2 on t1.k = t2.k and t1.s = t2.s "
                "group by t1.s order by t1.s"):
        got = ex.sql(sql, on_dev(ex, t1), right=on_dev(ex, t2))
        g = m2.groupby("s").agg(c=("v1", "size"), a=("v1", "sum"), b=("v2", "sum"))
        vals = list(got.values())
        assert vals[0].tolist() == g.index.tolist(), sql
        assert vals[1].tolist() == g.c.tolist() and vals[2].tolist() == g.a.tolist() and vals[3].tolist() == g.b.tolist()
    # LEFT JOIN USING: the unmatched FROM rows count, their k is the FROM table's
    got = ex.sql("select count(*) as c, sum(k) as sk from t2 left join t1 using (k)", on_dev(ex, t2),
                 right=on_dev(ex, t1))
    assert got["c"].tolist() == [n2] and got["sk"].tolist() == [int(t2["k"].sum())]


def test_sql_left_join_chain(ex, orc):
    """Chains with LEFT OUTER steps (the shape of the reference's fixture tests/sql/10.sql):
    INNER, then LEFT, then LEFT through a NULL-extended table's ON key (a NULL key matches
    nothing), or INNER through it (its NULL rows drop).  Aggregates over NULL-extended
    tables skip their NULL rows; pandas merges are the reference."""
    rng = np.random.default_rng(123)
    no, nl = 20_000, 60_000
    orders = {"o_okey": rng.permutation(no).astype(np.int64), "o_cust": rng.integers(0, 3000, no).astype(np.int64)}
    lines = {"l_okey": rng.integers(-500, no, nl).astype(np.int64), "l_qty": rng.integers(1, 50, nl).astype(np.int64)}
    cust = {"c_key": rng.permutation(3000)[:2000].astype(np.int64),  # a third of the customers missing
            "c_nation": rng.integers(0, 40, 2000).astype(np.int64)}
    nk = np.concatenate([np.arange(30), np.arange(10)])  # nations 30..39 missing, 0..9 twice
    nation = {"n_key": nk.astype(np.int64), "n_region": rng.integers(0, 5, len(nk)).astype(np.int64)}
    dl, do, dc, dn = (pd.DataFrame(t) for t in (lines, orders, cust, nation))
    right = [on_dev(ex, orders), on_dev(ex, cust), on_dev(ex, nation)]
    base = dl.merge(do, left_on="l_okey", right_on="o_okey").merge(dc, left_on="o_cust", right_on="c_key", how="left")
    for how in ("left", "inner"):
        m = base.merge(dn, left_on="c_nation", right_on="n_key", how=how)
        m = m[m.l_qty < 40]
        kw = "left join" if how == "left" else "join"
        got = ex.sql(f"""select l_qty, count(*) as c, count(c_nation) as cc, sum(c_nation) as sc,
                           count(n_region) as cr, sum(n_region) as sr, max(n_region) as mr
                         from lineitem join orders on l_okey = o_okey left join customer on o_cust = c_key
                         {kw} nation on c_nation = n_key where l_qty < 40 group by l_qty order by l_qty""",
                     on_dev(ex, lines), right=right)
        g = m.groupby("l_qty").agg(c=("l_qty", "size"), cc=("c_nation", "count"), sc=("c_nation", "sum"),
                                   cr=("n_region", "count"), sr=("n_region", "sum"), mr=("n_region", "max"))
        assert got["l_qty"].tolist() == g.index.tolist(), how
        for col in ("c", "cc", "sc", "cr", "sr"):
            assert got[col].tolist() == g[col].astype(np.int64).tolist(), (how, col)
        ok = g.mr.notna().to_numpy()
        assert got["mr"][ok].tolist() == g.mr[ok].astype(np.int64).tolist(), how
        if how == "inner":
            assert m.c_nation.notna().all()
    # global aggregates over a chain preserved from the FROM table; a scan keeps every row
    m = do.merge(dc, left_on="o_cust", right_on="c_key", how="left").merge(dn, left_on="c_nation", right_on="n_key",
                                                                          how="left")
    got = ex.sql("select count(*) as c, sum(n_region) as s, count(c_key) as k from orders "
                 "left join customer on o_cust = c_key left join nation on c_nation = n_key",
                 on_dev(ex, orders), right=right[1:])
    assert got["c"].tolist() == [len(m)] and got["s"].tolist() == [int(m.n_region.sum())]
    assert got["k"].tolist() == [int(m.c_key.notna().sum())]
    got = ex.sql("select o_okey from orders left join customer on o_cust = c_key left join nation on c_nation = n_key "
                 "where o_cust < 100 order by o_okey", on_dev(ex, orders), right=right[1:])
    assert got["o_okey"].tolist() == sorted(m.o_okey[m.o_cust < 100].tolist())
    # an INNER step on a NULL-extended key: its own table is never NULL (may be a group key)
    m = do.merge(dc, left_on="o_cust", right_on="c_key", how="left").merge(dn, left_on="c_nation", right_on="n_key")
    got = ex.sql("select n_region, count(*) as c, count(c_key) as k from orders left join customer on o_cust = c_key "
                 "join nation on c_nation = n_key group by n_region order by n_region", on_dev(ex, orders),
                 right=right[1:])
    g = m.groupby("n_region").agg(c=("o_okey", "size"), k=("c_key", "count"))
    assert got["n_region"].tolist() == g.index.tolist() and got["c"].tolist() == g.c.tolist()
    assert got["k"].tolist() == g.k.tolist()
    with pytest.raises(NutError, match="may only appear inside aggregates"):
        ex.sql("select n_region, count(*) from orders join customer on o_cust = c_key left join nation "
               "on c_nation = n_key group by n_region", on_dev(ex, orders), right=right[1:])


def test_sql_join_order_by_unprojected_column(ex, orc):
    """ORDER BY a column the SELECT list does not project, over an INNER join and over an
    INNER chain: the key column is gathered through the join index like a projection
    (it stayed bound to its source table and was read with joined-row ids).
    The joined rows outnumber the source table, so a wrong binding would also read out of
    range.  Ties keep the joined order (the sort is stable)."""
    orders, lines = tables(21, 5_000, 40_000, miss=0.1)
    j = joined(orc, lines, "l_okey", orders, "o_okey", "inner")
    got = ex.sql("select l_qty, l_price from lineitem join orders on l_okey = o_okey order by o_cust, l_price",
                 on_dev(ex, lines), right=on_dev(ex, orders))
    o = np.lexsort((j.l_price.to_numpy(), j.o_cust.to_numpy()))
    assert got["l_qty"].tolist() == j.l_qty.to_numpy()[o].tolist()
    assert got["l_price"].tolist() == j.l_price.to_numpy()[o].tolist()
    rng = np.random.default_rng(22)
    cust = {"c_key": np.arange(50, dtype=np.int64), "c_nation": rng.integers(0, 8, 50).astype(np.int64)}
    j["c_nation"] = cust["c_nation"][j.o_cust.to_numpy()]
    got = ex.sql("select l_qty from lineitem join orders on l_okey = o_okey join customer on o_cust = c_key "
                 "order by c_nation desc, l_qty limit 3000", on_dev(ex, lines),
                 right=[on_dev(ex, orders), on_dev(ex, cust)])
    o = np.lexsort((j.l_qty.to_numpy(), -j.c_nation.to_numpy()))
    assert got["l_qty"].tolist() == j.l_qty.to_numpy()[o][:3000].tolist()
    # a NULL-extended table's column may not order the rows (it would sort NULLs as 0)
    with pytest.raises(NutError, match="may only appear inside aggregates"):
        ex.sql("select o_okey from orders left join lineitem on o_okey = l_okey order by l_qty",
               on_dev(ex, orders), right=on_dev(ex, lines))
    with pytest.raises(NutError, match="may only appear inside aggregates"):
        ex.sql("select o_okey from orders join customer on o_cust = c_key left join lineitem on o_okey = l_okey "
               "order by l_qty", on_dev(ex, orders), right=[on_dev(ex, cust), on_dev(ex, lines)])
