"""GPU: typed tables from CREATE TABLE — the reference's own fixture
tests/sql/5.sql run verbatim over string columns, TPC-H Q1 over narrow / string / Date
columns, string predicates in both lowerings, narrow-type widening, Enum / Boolean, and
the string-misuse errors.  Ground truth: numpy over the same host data (exact: counts,
integer sums, dyadic or float32-widened values)."""
from pathlib import Path

import numpy as np
import pytest

from nutdb_amd import NutError
from nutdb_amd.table import Table

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).parent / "golden" / "sql"


def test_fixture5_verbatim(ex):
    """/root/reference/tests/sql/5.sql (copied as data to tests/golden/sql/5.sql), string
    constants and all, over one denormalised table."""
    rng = np.random.default_rng(55)
    n = 400_003
    modes = np.array(["MAIL", "SHIP", "AIR", "RAIL", "TRUCK", "FOB", "REG AIR"], dtype=object)
    prios = np.array(["1-URGENT", "2-HIGH", "3-MEDIUM", "4-NOT SPECIFIED", "5-LOW"], dtype=object)
    okey = rng.integers(0, 40, n)
    lkey = np.where(rng.random(n) < 0.6, okey, rng.integers(0, 40, n))
    mode = modes[rng.integers(0, len(modes), n)]
    prio = prios[rng.integers(0, len(prios), n)]
    ship = rng.integers(8000, 10000, n)
    commit = ship + rng.integers(-30, 30, n)
    receipt = ship + rng.integers(-30, 30, n)
    t = Table(ex, """CREATE TABLE orders (o_orderkey Int64, l_orderkey Int32, l_shipmode Dictionary(String),
        o_orderpriority String, l_shipdate Date, l_commitdate Date, l_receiptdate Date)""")
    t.append(o_orderkey=okey, l_orderkey=lkey.astype(np.int32), l_shipmode=mode, o_orderpriority=prio,
             l_shipdate=ship, l_commitdate=commit, l_receiptdate=receipt)
    assert t.nrows == n
    got = t.sql((GOLDEN / "5.sql").read_text(), group_hint=8)
    m = (okey == lkey) & np.isin(mode, ["MAIL", "SHIP"]) & (commit < receipt) & (ship < commit)
    hi_p = (prio == "1-URGENT") | (prio == "2-HIGH")
    assert got["l_shipmode"].tolist() == ["MAIL", "SHIP"]
    assert got["high_line_count"].tolist() == [int(np.sum(m & (mode == s) & hi_p)) for s in ("MAIL", "SHIP")]
    assert got["low_line_count"].tolist() == [int(np.sum(m & (mode == s) & ~hi_p)) for s in ("MAIL", "SHIP")]


def q1_table(ex, n, seed=11):
    rng = np.random.default_rng(seed)
    cols = dict(
        l_returnflag=np.array(["A", "N", "R"], dtype=object)[rng.integers(0, 3, n)],
        l_linestatus=np.array(["F", "O"], dtype=object)[rng.integers(0, 2, n)],
        l_quantity=rng.integers(1, 51, n).astype(np.int8),
        l_extendedprice=rng.integers(90000, 10494900, n) / 128.0,  # dyadic: exact sums
        l_discount=(rng.integers(0, 11, n) / 100.0).astype(np.float32),
        l_shipdate=rng.integers(8036, 10562, n),
    )
    t = Table(ex, """CREATE TABLE lineitem (l_returnflag Enum('A' = 65, 'N' = 78, 'R' = 82), l_linestatus String,
        l_quantity Int8, l_extendedprice Float64, l_discount Float32, l_shipdate Date)""")
    t.append(**cols)
    return t, cols


def test_q1_typed(ex):
    n = 300_007
    t, c = q1_table(ex, n)
    got = t.sql("""select l_returnflag, l_linestatus, sum(l_quantity) as sum_qty, sum(l_extendedprice) as base,
          avg(l_quantity) as avg_qty, max(l_discount) as max_disc, count(*) as count_order
        from lineitem where l_shipdate <= toDate('1998-12-01') - interval 90 day
        group by l_returnflag, l_linestatus order by l_returnflag desc, l_linestatus""", group_hint=6)
    m = c["l_shipdate"] <= 10471
    groups = sorted({(a, b) for a, b in zip(c["l_returnflag"][m], c["l_linestatus"][m])}, key=lambda g: (-ord(g[0]), g[1]))
    assert list(zip(got["l_returnflag"], got["l_linestatus"])) == groups
    for i, (a, b) in enumerate(groups):
        s = m & (c["l_returnflag"] == a) & (c["l_linestatus"] == b)
        assert got["sum_qty"][i] == int(np.sum(c["l_quantity"][s].astype(np.int64)))
        assert got["base"][i] == np.sum(c["l_extendedprice"][s])
        assert got["avg_qty"][i] == np.sum(c["l_quantity"][s].astype(np.int64)) / np.sum(s)
        assert got["max_disc"][i] == np.max(c["l_discount"][s].astype(np.float64))
        assert got["count_order"][i] == np.sum(s)


def test_string_predicates(ex):
    n = 100_003
    t, c = q1_table(ex, n, seed=3)
    rf, ls = c["l_returnflag"], c["l_linestatus"]
    cases = [
        ("l_returnflag = 'R'", rf == "R"),
        ("l_returnflag != 'R'", rf != "R"),
        ("l_linestatus in ('O', 'X')", ls == "O"),          # 'X' is in no row
        ("l_linestatus not in ('X')", np.ones(n, bool)),     # absent: every row
        ("l_linestatus = 'X'", np.zeros(n, bool)),
        ("'F' = l_linestatus", ls == "F"),
        ("l_returnflag = 'A' or l_linestatus = 'O'", (rf == "A") | (ls == "O")),  # expression mode
    ]
    for where, m in cases:
        got = t.sql(f"select count(*) as c from lineitem where {where}")
        assert got["c"].tolist() == [int(np.sum(m))], where
    got = t.sql("select l_linestatus, sum(case l_returnflag when 'A' then 1 when 'N' then 2 else 0 end) as s "
                "from lineitem group by l_linestatus order by l_linestatus")
    w = np.where(rf == "A", 1, np.where(rf == "N", 2, 0))
    assert got["l_linestatus"].tolist() == ["F", "O"]
    assert got["s"].tolist() == [int(np.sum(w[ls == "F"])), int(np.sum(w[ls == "O"]))]


@pytest.mark.parametrize("sql,frag", [
    ("select count(*) from lineitem where l_linestatus < 'G'", "ordering comparison"),
    ("select count(*) from lineitem where l_linestatus = 3", "compared with a number"),
    ("select count(*) from lineitem where l_quantity = 'a'", "non-string column"),
    ("select sum(l_linestatus) from lineitem", "only count"),
    ("select count(*) from lineitem where l_linestatus + 1 = 2 or l_quantity > 3", "= / != / IN"),
    ("select l_linestatus, count(*) from lineitem group by l_linestatus having l_linestatus > 0", "HAVING on the string key"),
    ("select l_linestatus from lineitem where l_linestatus = 'F' order by l_linestatus", "sorts"),
    ("select count(*) from lineitem where nosuch > 1", "no column 'nosuch'"),
])
def test_string_errors(ex, sql, frag):
    t, _ = q1_table(ex, 1000)
    with pytest.raises(NutError) as e:
        t.sql(sql)
    assert frag in str(e.value)


def test_widening_and_kinds(ex):
    t = Table(ex, "CREATE TABLE w (a Int8, b Int16, c Int32, d UInt8, e UInt16, f UInt32, g Boolean, h Float32, "
                  "i UInt64, k Int64)")
    a = np.array([-128, 127, -1, 0, 5], np.int8)
    b = np.array([-32768, 32767, -1, 0, 7], np.int16)
    c = np.array([-2**31, 2**31 - 1, -1, 0, 9], np.int32)
    d = np.array([255, 0, 1, 128, 3], np.uint8)
    e = np.array([65535, 0, 1, 32768, 3], np.uint16)
    f = np.array([2**32 - 1, 0, 1, 2**31, 3], np.uint32)
    g = np.array([1, 0, 7, 0, 1], np.uint8)
    h = np.array([0.1, -2.5, 3.0e38, -0.0, 1e-40], np.float32)
    i = np.array([2**63 - 1, 0, 1, 5, 3], np.uint64)
    k = np.arange(5, dtype=np.int64)
    t.append(a=a, b=b, c=c, d=d, e=e, f=f, g=g, h=h, i=i, k=k)
    # (at most 8 aggregates per plan)
    v1 = list(t.sql("select k, min(a), max(a), sum(b), sum(c), sum(d), max(f), sum(e), sum(g) "
                    "from w group by k order by k").values())
    v2 = list(t.sql("select k, min(h), max(h), max(i) from w group by k order by k").values())
    vals = v1 + v2[1:]
    assert vals[0].tolist() == k.tolist()
    assert vals[1].tolist() == a.astype(np.int64).tolist() and vals[2].tolist() == a.astype(np.int64).tolist()
    for got_col, src in zip(vals[3:8], (b, c, d, f, e)):
        assert got_col.tolist() == src.astype(np.int64).tolist()
    assert vals[8].tolist() == (g != 0).astype(np.int64).tolist()
    assert vals[9].tolist() == h.astype(np.float64).tolist()
    assert vals[11].tolist() == i.astype(np.int64).tolist()
    with pytest.raises(NutError) as err:
        t.append(i=np.array([2**63], np.uint64))
    assert "2^63" in str(err.value)
    t.append(k=np.array([9]))
    with pytest.raises(NutError) as err:  # rows are ragged until every column matches
        t.sql("select count(*) from w")
    assert "ragged" in str(err.value)


def test_enum_values(ex):
    t = Table(ex, "CREATE TABLE e (s Enum('lo' = 1, 'hi' = 9), v Int64)")
    t.append(s=["lo", "hi", "hi", "lo", "hi"], v=np.array([1, 2, 3, 4, 5]))
    got = t.sql("select s, sum(v) as sv from e where s != 'mid' group by s order by s")
    assert got["s"].tolist() == ["hi", "lo"] and got["sv"].tolist() == [10, 5]
    with pytest.raises(NutError) as err:
        t.append(s=["mid"])
    assert "not a value of its Enum" in str(err.value)


def test_tpch_q12_join_two_typed_tables(ex):
    """TPC-H Q12 as written (orders JOIN lineitem ON o_orderkey = l_orderkey) over two
    typed tables: string predicates on both sides, CASE over the other table's strings,
    string group keys decoded from their own table's dictionary (nut_table_execute2)."""
    rng = np.random.default_rng(12)
    no, nl = 50_000, 200_003
    prios = np.array(["1-URGENT", "2-HIGH", "3-MEDIUM", "4-NOT SPECIFIED", "5-LOW"], dtype=object)
    modes = np.array(["MAIL", "SHIP", "AIR", "RAIL", "TRUCK", "FOB", "REG AIR"], dtype=object)
    okey = rng.permutation(no).astype(np.int64) * 4 + 1
    prio = prios[rng.integers(0, len(prios), no)]
    lkey = np.where(rng.random(nl) < 0.9, okey[rng.integers(0, no, nl)], 2).astype(np.int64)
    mode = modes[rng.integers(0, len(modes), nl)]
    ship = rng.integers(8000, 10000, nl)
    commit = ship + rng.integers(-30, 30, nl)
    receipt = ship + rng.integers(-30, 30, nl)
    orders = Table(ex, "CREATE TABLE orders (o_orderkey Int64, o_orderpriority String)")
    orders.append(o_orderkey=okey, o_orderpriority=prio)
    lineitem = Table(ex, """CREATE TABLE lineitem (l_orderkey Int64, l_shipmode Dictionary(String),
        l_shipdate Date, l_commitdate Date, l_receiptdate Date)""")
    lineitem.append(l_orderkey=lkey, l_shipmode=mode, l_shipdate=ship, l_commitdate=commit, l_receiptdate=receipt)
    sql = """select l_shipmode,
        sum(case when o_orderpriority = '1-URGENT' or o_orderpriority = '2-HIGH' then 1 else 0 end) as high_line_count,
        sum(case when o_orderpriority <> '1-URGENT' and o_orderpriority <> '2-HIGH' then 1 else 0 end)
          as low_line_count
      from orders join lineitem on o_orderkey = l_orderkey
      where l_shipmode in ('MAIL', 'SHIP') and l_commitdate < l_receiptdate and l_shipdate < l_commitdate
      group by l_shipmode order by l_shipmode"""
    got = orders.sql(sql, group_hint=8, right=lineitem)
    pos = {k: i for i, k in enumerate(okey)}
    oi = np.array([pos.get(k, -1) for k in lkey])
    m = (oi >= 0) & np.isin(mode, ["MAIL", "SHIP"]) & (commit < receipt) & (ship < commit)
    lp = np.where(oi >= 0, prio[np.maximum(oi, 0)], "")
    hi = (lp == "1-URGENT") | (lp == "2-HIGH")
    assert got["l_shipmode"].tolist() == ["MAIL", "SHIP"]
    assert got["high_line_count"].tolist() == [int(np.sum(m & (mode == s) & hi)) for s in ("MAIL", "SHIP")]
    assert got["low_line_count"].tolist() == [int(np.sum(m & (mode == s) & ~hi)) for s in ("MAIL", "SHIP")]
    # a string key of the build side, grouped through the join
    got = lineitem.sql("select o_orderpriority, count(*) as c from lineitem join orders on l_orderkey = o_orderkey "
                       "group by o_orderpriority order by o_orderpriority", right=orders)
    assert got["o_orderpriority"].tolist() == sorted(prios.tolist())
    assert got["c"].tolist() == [int(np.sum((oi >= 0) & (lp == p))) for p in sorted(prios.tolist())]
    with pytest.raises(NutError, match="string keys"):
        lineitem.sql("select count(*) from lineitem join orders on l_shipmode = o_orderpriority", right=orders)


def test_scans_of_string_columns(ex):
    """FILTER scans over typed tables project dictionary columns: codes are gathered and
    decoded on output (single-column scans included)."""
    rng = np.random.default_rng(41)
    n = 100_003
    names = np.array(["ALPHA", "BRAVO", "CHARLIE", "DELTA"], dtype=object)
    s = names[rng.integers(0, 4, n)]
    k = rng.integers(0, 100, n)
    t = Table(ex, "CREATE TABLE t (s String, k Int64, e Enum('x' = 1, 'y' = 2))")
    e = np.array(["x", "y"], dtype=object)[rng.integers(0, 2, n)]
    t.append(s=s, k=k, e=e)
    got = t.sql("select s from t where s = 'BRAVO' or s = 'DELTA'")
    assert got["s"].tolist() == s[(s == "BRAVO") | (s == "DELTA")].tolist()
    got = t.sql("select k, s, e from t where k < 3 and e = 'y' limit 50")
    m = (k < 3) & (e == "y")
    assert got["k"].tolist() == k[m][:50].tolist() and got["s"].tolist() == s[m][:50].tolist()
    assert got["e"].tolist() == e[m][:50].tolist()
    assert t.sql("select s from t")["s"].tolist() == s.tolist()


def _like(v, pat, ci=False):
    import re
    rx = ""
    i = 0
    while i < len(pat):
        ch = pat[i]
        if ch == "\\" and i + 1 < len(pat):
            rx += re.escape(pat[i + 1])
            i += 2
            continue
        rx += ".*" if ch == "%" else "." if ch == "_" else re.escape(ch)
        i += 1
    return re.fullmatch(rx, v, re.S | (re.I if ci else 0)) is not None


def test_like_on_dictionary_columns(ex):
    """[NOT] [I]LIKE over String / Enum columns: evaluated once per dictionary string (a
    per-code match table), in scans, aggregates and joins' pushed WHERE."""
    rng = np.random.default_rng(43)
    n = 200_003
    types = np.array(["STANDARD POLISHED BRASS", "SMALL BRUSHED TIN", "LARGE PLATED BRASS", "ECONOMY ANODIZED STEEL",
                      "PROMO BURNISHED COPPER", "MEDIUM POLISHED brass", "50%_OFF", "50X_OFF"], dtype=object)
    ty = types[rng.integers(0, len(types), n)]
    size = rng.integers(1, 50, n)
    t = Table(ex, "CREATE TABLE part (p_type String, p_size Int64, p_e Enum('red' = 1, 'green' = 2))")
    pe = np.array(["red", "green"], dtype=object)[rng.integers(0, 2, n)]
    t.append(p_type=ty, p_size=size, p_e=pe)
    for where, m in [
        ("p_type like '%BRASS'", np.array([_like(v, "%BRASS") for v in ty])),
        ("p_type ilike '%brass'", np.array([_like(v, "%brass", True) for v in ty])),
        ("p_type not like 'S%'", np.array([not _like(v, "S%") for v in ty])),
        ("p_type like '_MALL%' or p_size > 45", np.array([_like(v, "_MALL%") for v in ty]) | (size > 45)),
        ("p_type like '50\\\\%\\\\_OFF'", ty == "50%_OFF"),
        ("p_type like 'NOTHING%'", np.zeros(n, bool)),
        ("p_e like 'gr%'", pe == "green"),
    ]:
        got = t.sql(f"select count(*) as c, sum(p_size) as s from part where {where}")
        assert got["c"].tolist() == [int(m.sum())] and got["s"].tolist() == [int(size[m].sum())], where
    got = t.sql("select p_size from part where p_type like '%TIN' and p_size < 10")
    assert got["p_size"].tolist() == size[(ty == "SMALL BRUSHED TIN") & (size < 10)].tolist()
    with pytest.raises(NutError, match="LIKE needs a string column"):
        t.sql("select count(*) from part where p_size like '1%'")


def test_like_through_a_join(ex):
    """LIKE on the other table's dictionary column: pushed below the join alone, and kept
    above it inside a cross-table OR (the column is gathered through the join index)."""
    rng = np.random.default_rng(47)
    names = np.array(["ACME BOLT", "ACME NUT", "ZED BOLT", "ZED GEAR"], dtype=object)
    nparts, nl = 1000, 50_003
    pkey = rng.permutation(nparts).astype(np.int64)
    pname = names[rng.integers(0, 4, nparts)]
    part = Table(ex, "CREATE TABLE part (p_key Int64, p_name String)")
    part.append(p_key=pkey, p_name=pname)
    lk = rng.integers(0, nparts, nl).astype(np.int64)
    qty = rng.integers(1, 50, nl).astype(np.int64)
    li = Table(ex, "CREATE TABLE lineitem (l_part Int64, l_qty Int64)")
    li.append(l_part=lk, l_qty=qty)
    nm = dict(zip(pkey.tolist(), pname.tolist()))
    ln = np.array([nm[k] for k in lk.tolist()], dtype=object)
    for where, m in [("p_name like 'ACME%'", np.array([v.startswith("ACME") for v in ln])),
                     ("p_name like '%BOLT' or l_qty > 45", np.array([v.endswith("BOLT") for v in ln]) | (qty > 45))]:
        got = li.sql(f"select count(*) as c, sum(l_qty) as s from lineitem join part on l_part = p_key where {where}",
                     right=part)
        assert got["c"].tolist() == [int(m.sum())] and got["s"].tolist() == [int(qty[m].sum())], where


def test_like_large_dictionaries(ex):
    """LIKE is a per-code byte table over the dictionary (nut_prog LOOKUP): thousands of
    matching strings, two LIKEs in one program, `_` as one UTF-8 character, and an Enum
    whose ids are too sparse for a table (ORed equalities)."""
    rng = np.random.default_rng(53)
    n = 300_007
    words = np.array([f"W{i:05d}-{'é' if i % 3 == 0 else 'e'}nd" for i in range(6000)], dtype=object)
    w = words[rng.integers(0, len(words), n)]
    x = rng.integers(0, 100, n)
    big = np.array(["lo", "hi", "mid"], dtype=object)[rng.integers(0, 3, n)]
    t = Table(ex, "CREATE TABLE t (w String, x Int64, e Enum('lo' = 7, 'hi' = 100000000, 'mid' = 4000000000))")
    t.append(w=w, x=x, e=big)
    cases = [
        ("w like 'W0%'", np.array([v.startswith("W0") for v in w])),  # ~4000 matching strings
        ("w like '%_nd' and w not like 'W1%'", np.array([not v.startswith("W1") for v in w])),
        ("w like 'W____0-_nd'", np.array([_like(v, "W____0-_nd") for v in w])),  # é is one `_`
        ("w like '%é%' or x < 3", np.array(["é" in v for v in w]) | (x < 3)),
        ("e like '%i%'", (big == "hi") | (big == "mid")),
        ("e like 'l_'", big == "lo"),
        ("e like 'zz%'", np.zeros(n, bool)),
    ]
    for where, m in cases:
        assert m.any() or "zz" in where
        got = t.sql(f"select count(*) as c, sum(x) as s from t where {where}")
        assert got["c"].tolist() == [int(m.sum())] and got["s"].tolist() == [int(x[m].sum())], where
    got = t.sql("select x from t where w like 'W00___-é%' limit 100000")
    m = np.array([_like(v, "W00___-é%") for v in w])
    assert m.sum() > 0 and got["x"].tolist() == x[m].tolist()


def test_join_chain_typed_tables(ex):
    """lineitem JOIN orders JOIN customer over typed tables (nut_table_executen): LIKE /
    IN / = on the strings of every table, string GROUP BY keys and string projections
    decoded from their own table's dictionary; string JOIN keys are rejected."""
    rng = np.random.default_rng(61)
    nc, no, nl = 2000, 20_000, 100_003
    segs = np.array(["AUTOMOBILE", "BUILDING", "FURNITURE", "HOUSEHOLD", "MACHINERY"], dtype=object)
    prios = np.array(["1-URGENT", "2-HIGH", "3-MEDIUM", "4-NOT SPECIFIED", "5-LOW"], dtype=object)
    modes = np.array(["MAIL", "SHIP", "AIR", "RAIL", "TRUCK"], dtype=object)
    ckey = rng.permutation(nc).astype(np.int64) + 10
    seg = segs[rng.integers(0, len(segs), nc)]
    okey = rng.permutation(no).astype(np.int64) * 3
    ocust = ckey[rng.integers(0, nc, no)]
    ocust[:50] = -5  # no customer
    prio = prios[rng.integers(0, len(prios), no)]
    lkey = okey[rng.integers(0, no, nl)]
    qty = rng.integers(1, 51, nl).astype(np.int64)
    mode = modes[rng.integers(0, len(modes), nl)]
    customer = Table(ex, "CREATE TABLE customer (c_custkey Int64, c_mktsegment String)")
    customer.append(c_custkey=ckey, c_mktsegment=seg)
    orders = Table(ex, "CREATE TABLE orders (o_orderkey Int64, o_custkey Int64, o_orderpriority String)")
    orders.append(o_orderkey=okey, o_custkey=ocust, o_orderpriority=prio)
    lineitem = Table(ex, "CREATE TABLE lineitem (l_orderkey Int64, l_quantity Int64, l_shipmode Dictionary(String))")
    lineitem.append(l_orderkey=lkey, l_quantity=qty, l_shipmode=mode)
    opos = {k: i for i, k in enumerate(okey.tolist())}
    cpos = {k: i for i, k in enumerate(ckey.tolist())}
    oi = np.array([opos[k] for k in lkey.tolist()])
    ci = np.array([cpos.get(k, -1) for k in ocust[oi].tolist()])
    ok = ci >= 0
    lseg = np.where(ok, seg[np.maximum(ci, 0)], "")
    lprio = prio[oi]
    frm = "from lineitem join orders on l_orderkey = o_orderkey join customer on o_custkey = c_custkey"
    got = lineitem.sql(f"""select c_mktsegment, count(*) as c, sum(l_quantity) as s {frm}
        where (o_orderpriority like '1-%' or o_orderpriority = '2-HIGH') and l_shipmode in ('MAIL', 'SHIP')
        group by c_mktsegment order by c_mktsegment""", group_hint=8, joined=[orders, customer])
    m = ok & np.isin(lprio, ["1-URGENT", "2-HIGH"]) & np.isin(mode, ["MAIL", "SHIP"])
    want = sorted(set(lseg[m].tolist()))
    assert got["c_mktsegment"].tolist() == want
    assert got["c"].tolist() == [int(np.sum(m & (lseg == s))) for s in want]
    assert got["s"].tolist() == [int(qty[m & (lseg == s)].sum()) for s in want]
    got = lineitem.sql(f"""select l_shipmode, c_mktsegment, o_orderpriority, l_quantity {frm}
        where l_quantity > 47 and c_mktsegment like 'B%'""", joined=[orders, customer])
    m = ok & (qty > 47) & (lseg == "BUILDING")
    rows = sorted(zip(got["l_shipmode"].tolist(), got["c_mktsegment"].tolist(), got["o_orderpriority"].tolist(),
                      got["l_quantity"].tolist()))
    assert rows == sorted(zip(mode[m].tolist(), lseg[m].tolist(), lprio[m].tolist(), qty[m].tolist()))
    with pytest.raises(NutError, match="string keys"):
        lineitem.sql("select count(*) from lineitem join orders on l_orderkey = o_orderkey "
                     "join customer on o_orderpriority = c_mktsegment", joined=[orders, customer])


def test_join_string_columns_of_two_tables_rejected(ex):
    """Each typed table has its own dictionary, so a String column of one table never
    compares with one of another (USING (k, s) compared codes of two
    dictionaries and returned wrong rows).  USING / ON / WHERE forms are rejected with a
    message naming the cause; an integer USING key and strings against constants run."""
    rng = np.random.default_rng(48)
    n1, n2 = 500, 4000
    t1 = Table(ex, "CREATE TABLE t1 (k Int64, s String, v Int64)")
    t1.append(k=np.arange(n1, dtype=np.int64), s=np.array(["a", "b"], dtype=object)[rng.integers(0, 2, n1)],
              v=rng.integers(0, 9, n1).astype(np.int64))
    t2 = Table(ex, "CREATE TABLE t2 (k Int64, s String, w Int64)")
    s2 = np.array(["b", "a", "c"], dtype=object)[rng.integers(0, 3, n2)]  # first-seen order differs
    k2 = rng.integers(0, n1, n2).astype(np.int64)
    t2.append(k=k2, s=s2, w=rng.integers(0, 9, n2).astype(np.int64))
    for sql in ("select count(*) from t1 join t2 using (k, s)",
                "select count(*) from t1 join t2 on t1.k = t2.k and t1.s = t2.s",
                "select count(*) from t1 join t2 on t1.k = t2.k where t1.s = t2.s"):
        with pytest.raises(NutError, match="dictionaries differ"):
            t1.sql(sql, right=t2)
    got = t1.sql("select count(*) as c from t1 join t2 using (k) where t2.s = 'c'", right=t2)
    assert got["c"].tolist() == [int((s2 == "c").sum())]


def test_fixture1_tpch_q1_with_joins_flattened(ex):
    """The reference fixture tests/sql/1.sql (TPC-H Q1 with the Q2-style join predicates
    flattened into one table's WHERE: p_partkey = ps_partkey, p_type LIKE '%BRASS',
    r_name = 'EUROPE', ...) over one denormalised typed table.  Its ORDER BY's first key
    s_acctbal is neither grouped nor aggregated — an error in SQL — and is dropped; the rest
    runs verbatim: 10 SELECT items, three AVGs sharing count(*) (6 aggregates)."""
    from helpers import F64_SUM_RTOL, rel_err
    sql = (GOLDEN / "1.sql").read_text().replace("s_acctbal desc,", "")
    rng = np.random.default_rng(101)
    n = 400_009
    types = np.array(["SMALL BRASS", "LARGE BRASS", "PLATED STEEL", "BRASS TIN"], dtype=object)
    regions = np.array(["EUROPE", "ASIA", "AMERICA"], dtype=object)
    pk = rng.integers(0, 50, n)
    sk = rng.integers(0, 50, n)
    nk = rng.integers(0, 25, n)
    c = dict(l_returnflag=rng.integers(0, 3, n), l_linestatus=rng.integers(0, 2, n),
             l_quantity=rng.integers(1, 51, n).astype(np.float64), l_extendedprice=rng.integers(90000, 10494900, n) / 100,
             l_discount=rng.integers(0, 11, n) / 100, l_tax=rng.integers(0, 9, n) / 100,
             l_shipdate=rng.integers(8036, 10562, n), p_partkey=pk,
             ps_partkey=np.where(rng.random(n) < 0.7, pk, pk + 1), s_suppkey=sk,
             ps_suppkey=np.where(rng.random(n) < 0.8, sk, sk + 3), p_size=rng.integers(10, 20, n),
             p_type=types[rng.integers(0, 4, n)], s_nationkey=nk,
             n_nationkey=np.where(rng.random(n) < 0.9, nk, nk + 1), r_name=regions[rng.integers(0, 3, n)])
    t = Table(ex, """CREATE TABLE lineitem (l_returnflag Int64, l_linestatus Int64, l_quantity Float64,
        l_extendedprice Float64, l_discount Float64, l_tax Float64, l_shipdate Date, p_partkey Int64,
        ps_partkey Int64, s_suppkey Int64, ps_suppkey Int64, p_size Int64, p_type String, s_nationkey Int64,
        n_nationkey Int64, r_name String)""")
    t.append(**c)
    got = t.sql(sql, group_hint=6)
    m = ((c["l_shipdate"] <= 10561 - 10) & (c["p_partkey"] == c["ps_partkey"]) & (c["s_suppkey"] == c["ps_suppkey"])
         & (c["p_size"] == 15) & np.array([s.endswith("BRASS") for s in c["p_type"]])
         & (c["s_nationkey"] == c["n_nationkey"]) & (c["l_shipdate"] > 9204) & (c["r_name"] == "EUROPE"))
    keys = sorted({(a, b) for a, b in zip(c["l_returnflag"][m], c["l_linestatus"][m])})
    assert list(zip(got["l_returnflag"], got["l_linestatus"])) == keys and len(keys) == 6
    price, disc, tax, qty = c["l_extendedprice"], c["l_discount"], c["l_tax"], c["l_quantity"]
    for i, (a, b) in enumerate(keys):
        s = m & (c["l_returnflag"] == a) & (c["l_linestatus"] == b)
        want = {"sum_qty": qty[s].sum(), "sum_base_price": price[s].sum(),
                "sum_disc_price": (price[s] * (1 - disc[s])).sum(),
                "sum_charge": (price[s] * (1 - disc[s]) * (1 + tax[s])).sum(),
                "avg_qty": qty[s].mean(), "avg_price": price[s].mean(), "avg_disc": disc[s].mean()}
        for k, w in want.items():
            assert rel_err(np.array([got[k][i]]), np.array([w])) <= F64_SUM_RTOL, (k, a, b)
        assert got["count_order"][i] == int(s.sum())
