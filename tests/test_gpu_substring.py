"""substring over dictionary strings on the GPU, against pandas.

The reference's fixture tests/sql/9.sql (TPC-H Q22) reads `substring(c_phone, 1, 2)` in a
derived table's projection, its WHERE (an IN list) and a scalar subquery's WHERE, next to a
NOT EXISTS over orders, and groups the derived rows by it.  The executor maps the string
column's dictionary codes to their substrings' codes (one MAP node of the expression kernel:
a gather from a per-code int64 table), so the kernels never touch the bytes.  Semantics are
ClickHouse's byte `substring`: 1-based offset, a negative offset counts from the end, offset
0 gives '', a negative length stops that many bytes before the end.  Counts and keys
bit-exact; f64 sums within F64_SUM_RTOL.
"""
from pathlib import Path

import numpy as np
import pandas as pd
import pytest

from helpers import F64_SUM_RTOL, rel_err
from nutdb_amd.table import Table

pytestmark = pytest.mark.gpu

SQL = Path(__file__).parent / "golden" / "sql"


def ch_substring(s: str, off: int, ln=None) -> str:
    """ClickHouse `substring(s, off[, len])` over bytes (ASCII here): the window [w0, w1)
    starts at off - 1 (off > 0) or |off| before the end (off < 0), is clipped to the string."""
    n = len(s)
    if off == 0:
        return ""
    w0 = off - 1 if off > 0 else n + off
    w1 = n if ln is None else (w0 + ln if ln >= 0 else n + ln)
    b, e = max(0, min(w0, n)), min(w1, n)
    return s[b:e] if e > b else ""


def test_ch_substring_restatement():
    """the test's own restatement on the cases ClickHouse documents"""
    assert ch_substring("Hello, world!", 1, 5) == "Hello"
    assert ch_substring("Hello, world!", -6) == "world!"
    assert ch_substring("Hello, world!", 8, -1) == "world"
    assert ch_substring("abc", 0, 2) == "" and ch_substring("abc", 5) == ""
    assert ch_substring("abc", -9, 2) == "" and ch_substring("abc", -4, 2) == "a" and ch_substring("abc", -9) == "abc"


def phones(rng, n):
    cc = rng.integers(10, 35, n)
    return np.array([f"{c}-{rng.integers(100, 999)}-{rng.integers(100, 999)}-{rng.integers(1000, 9999)}"
                     for c in cc], dtype=object)


def test_fixture9_q22(ex):
    """TPC-H Q22 as written (tests/sql/9.sql): substring in the derived table's projection,
    its WHERE and the scalar subquery's WHERE; NOT EXISTS over orders; GROUP BY cntrycode."""
    rng = np.random.default_rng(9)
    nc, no = 150_000, 300_000
    cust = {"c_custkey": rng.permutation(nc * 2)[:nc].astype(np.int64), "c_phone": phones(rng, nc),
            "c_acctbal": np.round(rng.uniform(-999.99, 9999.99, nc), 2)}
    orders = {"o_custkey": rng.choice(cust["c_custkey"], no).astype(np.int64)}
    t = Table(ex, "CREATE TABLE customer (c_custkey Int64, c_phone String, c_acctbal Float64)")
    t.append(**cust)
    o = Table(ex, "CREATE TABLE orders (o_custkey Int64)")
    o.append(**orders)
    got = t.sql((SQL / "9.sql").read_text(), joined=[o])
    d = pd.DataFrame(cust)
    d["cntry"] = d.c_phone.str[:2]
    codes = ["13", "31", "23", "29", "30", "18", "17"]
    avg = d.c_acctbal[(d.c_acctbal > 0) & d.cntry.isin(codes)].mean()
    m = d[d.cntry.isin(codes) & (d.c_acctbal > avg) & ~d.c_custkey.isin(set(orders["o_custkey"]))]
    g = m.groupby("cntry").agg(numcust=("c_acctbal", "size"), totacctbal=("c_acctbal", "sum")).sort_index()
    assert len(g) == 7 and g.numcust.sum() > 1000
    assert list(got["cntrycode"]) == g.index.tolist()
    assert got["numcust"].tolist() == g.numcust.tolist()
    assert rel_err(np.asarray(got["totacctbal"]), g.totacctbal.to_numpy()) < F64_SUM_RTOL


@pytest.mark.parametrize("off,ln", [(1, 2), (-3, None), (2, -2), (0, 3), (7, 50), (-40, 3), (4, 0)])
def test_substring_group_by_semantics(ex, off, ln):
    """GROUP BY substring(s, off[, len]) with count and sum: every offset / length form"""
    rng = np.random.default_rng(100 + off)
    n = 80_000
    words = np.array(["alpha", "beta", "gamma", "delta", "epsilon", "zeta", "eta", "theta", "x", ""], dtype=object)
    s = np.array([w + str(i) for w, i in zip(words[rng.integers(0, len(words), n)], rng.integers(0, 30, n))],
                 dtype=object)
    v = rng.integers(-1000, 1000, n).astype(np.int64)
    t = Table(ex, "CREATE TABLE tb (s String, v Int64)")
    t.append(s=s, v=v)
    arg = f"{off}" if ln is None else f"{off}, {ln}"
    got = t.sql(f"select substring(s, {arg}) as sub, count(*) as c, sum(v) as sv from tb group by sub order by sub")
    d = pd.DataFrame({"s": s, "v": v})
    d["sub"] = d.s.map(lambda x: ch_substring(x, off, ln))
    g = d.groupby("sub").agg(c=("v", "size"), sv=("v", "sum")).sort_index()
    assert list(got["sub"]) == g.index.tolist()
    assert got["c"].tolist() == g.c.tolist() and got["sv"].tolist() == g.sv.tolist()


def test_substring_where_projection_and_constants(ex):
    """WHERE substring(..) = / IN / != constants (one only a substring has, one no string
    has), a substring compared with its own column, and a substring projection"""
    rng = np.random.default_rng(5)
    n = 50_000
    pool = np.array(["ab", "abc", "abcd", "b", "bcd", "cd", "zz9"], dtype=object)
    s = pool[rng.integers(0, len(pool), n)]
    v = np.arange(n, dtype=np.int64)
    t = Table(ex, "CREATE TABLE tb (s String, v Int64)")
    t.append(s=s, v=v)
    d = pd.DataFrame({"s": s, "v": v})
    sub2 = d.s.str[:2]
    cases = [
        ("substring(s, 1, 2) = 'ab'", sub2 == "ab"),
        ("substring(s, 1, 2) in ('bc', 'zz', 'qq')", sub2.isin(["bc", "zz", "qq"])),
        ("'cd' != substring(s, 1, 2)", sub2 != "cd"),
        ("substring(s, 1, 2) = s", sub2 == d.s),
        ("substring(s, 2) = 'bcd'", d.s.str[1:] == "bcd"),
        ("substring(s, 1, 1) = 'nothing'", pd.Series(False, index=d.index)),
    ]
    for where, mask in cases:
        got = t.sql(f"select count(*) as c, sum(v) as sv from tb where {where}")
        assert got["c"].tolist() == [int(mask.sum())], where
        assert got["sv"].tolist() == [int(d.v[mask].sum())], where
    got = t.sql("select v, substring(s, -2) as tail from tb where v < 1000 order by v")
    assert got["v"].tolist() == list(range(1000))
    assert list(got["tail"]) == [x[-2:] for x in s[:1000]]
