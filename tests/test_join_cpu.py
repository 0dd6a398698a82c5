"""CPU: the hash-join oracle (oracle/oracle.py join_i64) against a brute-force nested
loop on small inputs, and the known answers of the join types (include/nutexec.h)."""
import numpy as np
import pytest

from oracle.oracle import join_i64


def brute(build, probe, how):
    pi, bi = [], []
    for r, k in enumerate(probe):
        hits = [j for j, b in enumerate(build) if b == k]
        if how == "inner":
            pi += [r] * len(hits)
            bi += hits
        elif how == "left":
            pi += [r] * max(len(hits), 1)
            bi += hits if hits else [-1]
        elif how == "semi" and hits:
            pi.append(r)
            bi.append(-1)
        elif how == "anti" and not hits:
            pi.append(r)
            bi.append(-1)
    return np.array(pi, dtype=np.int64), np.array(bi, dtype=np.int64)


def test_join_known_answers():
    b = np.array([5, 3, 5, 7])
    p = np.array([5, 1, 7, 3, 5])
    assert [x.tolist() for x in join_i64(b, p, "inner")] == [[0, 0, 2, 3, 4, 4], [0, 2, 3, 1, 0, 2]]
    assert [x.tolist() for x in join_i64(b, p, "left")] == [[0, 0, 1, 2, 3, 4, 4], [0, 2, -1, 3, 1, 0, 2]]
    assert join_i64(b, p, "semi")[0].tolist() == [0, 2, 3, 4]
    assert join_i64(b, p, "anti")[0].tolist() == [1]


@pytest.mark.parametrize("how", ["inner", "left", "semi", "anti"])
@pytest.mark.parametrize("seed", range(6))
def test_join_oracle_vs_nested_loop(how, seed):
    rng = np.random.default_rng(seed)
    nb, npr = [(0, 5), (5, 0), (30, 40), (64, 200), (200, 64), (1, 1)][seed]
    b = rng.integers(-8, 8, nb).astype(np.int64)
    p = rng.integers(-10, 10, npr).astype(np.int64)
    got, want = join_i64(b, p, how), brute(b.tolist(), p.tolist(), how)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


# ------------------------------------------------------------------ SQL JOIN lowering
JQ = "select o_cust, count(*) as c, sum(l_qty) as s from orders {} lineitem on o_okey = l_okey group by o_cust"


@pytest.mark.parametrize("kw,typ,right,mode", [
    ("join", "inner", False, "fused"), ("inner join", "inner", False, "fused"),
    ("left join", "left", False, "compiled"), ("left outer join", "left", False, "compiled"),
    ("right join", "left", True, "compiled"), ("left semi join", "semi", False, "fused"),
    ("right semi join", "semi", True, "fused"), ("left anti join", "anti", False, "fused"),
    ("right anti join", "anti", True, "fused")])
def test_sql_join_lowering(kw, typ, right, mode):
    from nutdb_amd.sql import Plan
    d = Plan(JQ.format(kw)).describe()
    assert d["join"] == {"type": typ, "right": right, "table": "lineitem", "aliases": ["", ""],
                         "on": ["o_okey", "l_okey"]}
    assert d["table"] == "orders" and d["mode"] == mode  # outer joins mask aggregates: expression mode
    assert set(d["columns"]) == {"o_okey", "l_okey", "o_cust", "l_qty"}


def test_sql_full_join_lowers_to_expression_mode():
    """FULL OUTER JOIN: both tables NULL-extended, aggregates masked per side (expression mode)."""
    from nutdb_amd.sql import Plan
    d = Plan("select count(*), sum(l_qty) from orders full outer join lineitem on o_okey = l_okey").describe()
    assert d["join"]["type"] == "full" and d["join"]["right"] is False
    assert d["mode"] == "compiled"


def test_sql_no_join_has_no_join_key():
    from nutdb_amd.sql import Plan
    assert "join" not in Plan("select k, count(*) from t group by k").describe()


@pytest.mark.parametrize("sql,msg", [
    ("select count(*) from a full join b on x = y and u = v", "INNER only"),
    ("select count(*) from a join b on x < y", "needs an equality of two columns"),
    ("select count(*) from a right join b on x = y and u < v", "INNER, LEFT, SEMI and ANTI"),
    ("select count(*) from a left join b on x = y and u = v", "INNER only"),
    ("select count(*) from a left semi join b using (x, y)", "INNER only"),
    ("select count(*) from a join b using (x) join c using (x)", "USING in a chain"),
    ("select count(*) from a join b on x = y right anti join c on y = z", "steps only"),
    ("select count(*) from a join (select x from b) on x = y", "must be a table"),
    # FULL OUTER ... USING (u): an unqualified u would be COALESCE(a.u, b.u)
    ("select count(u), sum(u) from a full outer join b using (u)", "FULL OUTER JOIN ... USING"),
    ("select u, count(*) from a full join b using (u) group by u", "FULL OUTER JOIN ... USING")])
def test_sql_join_rejections(sql, msg):
    from nutdb_amd import NutError
    from nutdb_amd.sql import Plan
    with pytest.raises(NutError, match=msg):
        Plan(sql)


def test_count_star_and_count_column_stay_apart():
    """count(l_qty) and count(*) are one aggregate without a join, two under an outer join
    (the NULL-extended rows count for * only)."""
    from nutdb_amd.sql import Plan
    d = Plan("select o_cust, count(*), count(l_qty) from orders left join lineitem on o_okey = l_okey "
             "group by o_cust").describe()
    assert len(d["aggs"]) == 2


@pytest.mark.parametrize("how", ["inner", "left", "semi", "anti"])
@pytest.mark.parametrize("nb,npr", [(0, 7), (7, 0), (300, 1000), (20_000, 200_000)])
def test_c_join_oracle_matches_numpy(how, nb, npr):
    """oracle.c orc_join_i64 (the bench's CPU baseline) against the numpy oracle; the C
    join leaves the build rows of one probe row unordered, so pairs compare sorted."""
    from oracle.oracle import join_i64_c
    rng = np.random.default_rng(nb + npr)
    b = rng.integers(-500, 500, nb).astype(np.int64)
    p = rng.integers(-600, 600, npr).astype(np.int64)
    a, c = join_i64(b, p, how), join_i64_c(b, p, how)
    assert np.all(c[0][1:] >= c[0][:-1])
    o = np.lexsort((c[1], c[0]))
    assert np.array_equal(a[0], c[0][o]) and np.array_equal(a[1], c[1][o])


def test_sql_join_qualified_names():
    from nutdb_amd.sql import Plan
    d = Plan("select o.cust, count(*) from orders as o join lineitem as l on o.okey = l.okey "
             "group by o.cust").describe()
    assert d["join"]["on"] == ["o.okey", "l.okey"] and d["keys"] == ["o.cust"]
    # without a JOIN the qualifier is dropped, as before
    assert Plan("select t.a from t where t.a > 3").describe()["columns"] == ["a"]


def test_sql_join_chain_lowering():
    from nutdb_amd.sql import Plan
    d = Plan("select c_nation, count(*) from lineitem join orders on l_okey = o_okey join customer on "
             "o_cust = c_key group by c_nation").describe()
    assert d["joins"] == [{"table": "orders", "type": "inner", "on": ["l_okey", "o_okey"]},
                          {"table": "customer", "type": "inner", "on": ["o_cust", "c_key"]}]
    # LEFT OUTER steps (fixture 10's chain shape); other types and several LEFT keys are not
    d = Plan("select count(*) from a join b on x = y left join c on y = z left join d on z = w").describe()
    assert [j["type"] for j in d["joins"]] == ["inner", "left", "left"]
    # aggregates over a chain with a LEFT step take expression mode (NULL-row masks)
    assert Plan("select x, sum(z) from a join b on x = y left join c on y = z group by x").describe()["mode"] == "compiled"
    from nutdb_amd import NutError
    # RIGHT / FULL OUTER and LEFT SEMI / ANTI steps too; not RIGHT SEMI / ANTI or ASOF
    d = Plan("select count(*) from a join b on x = y right join c on y = z full join d on z = w "
             "left semi join e on w = v left anti join f on w = u").describe()
    assert [j["type"] for j in d["joins"]] == ["inner", "right", "full", "semi", "anti"]
    with pytest.raises(NutError, match="steps only"):
        Plan("select count(*) from a join b on x = y right semi join c on y = z")
    with pytest.raises(NutError, match="several key columns: INNER only"):
        Plan("select count(*) from a join b on x = y left join c on y = z and x = w")


def test_sql_join_using_and_multi_key_lowering():
    """USING (u): the FROM table's u = the source's u, an unqualified u elsewhere is the
    preserved table's; further key columns (USING (a, b), ON a = b AND c = d) join on the
    first and filter the pairs by the rest above the join (INNER)."""
    from nutdb_amd.sql import Plan
    d = Plan("select k, count(*) from orders join lineitem using (k) group by k").describe()
    assert d["join"]["on"] == ["orders.k", "lineitem.k"] and d["keys"] == ["orders.k"]
    d = Plan("select sum(v) from orders as o right join lineitem as l using (k) where k > 3").describe()
    assert d["join"]["on"] == ["o.k", "l.k"] and d["join"]["right"] is True
    assert "l.k" in d["columns"] and "k" not in d["columns"]
    d = Plan("select count(*) from a join b using (x, y)").describe()
    assert d["join"]["on"] == ["a.x", "b.x"] and d["mode"] == "compiled" and d["where_expr"] == "(a.y = b.y)"
    d = Plan("select count(*) from a join b on a.x = b.x and a.y = b.y where a.z > 1").describe()
    assert d["join"]["on"] == ["a.x", "b.x"] and d["where_expr"] == "((a.z > 1) and (a.y = b.y))"
    d = Plan("select count(*) from l join o on lk = ok join c on oc = ck and on_ = cn").describe()
    assert d["joins"][1] == {"table": "c", "type": "inner", "on": ["oc", "ck"]} and d["where_expr"] == "(on_ = cn)"


# ---- grouped derived tables, CTEs, JOIN ON filters
from nutdb_amd._lib import NutError  # noqa: E402
from nutdb_amd.sql import Plan  # noqa: E402

Q13_CTE = ("with c_orders as (select c_custkey, count(o_orderkey) as c_count from customer left outer join orders "
           "on c_custkey = o_custkey and o_comment not like '%special%requests%' group by c_custkey) "
           "select c_count, count(*) as custdist from c_orders group by c_count order by custdist desc, c_count desc")


def test_plan_cte_materialized_with_on_filter():
    d = Plan(Q13_CTE).describe()
    assert d["kind"] == "groupby" and d["table"] == "c_orders" and d["keys"] == ["c_count"]
    assert d["derived_columns"] == ["c_count"]
    inner = d["derived"]
    assert inner["kind"] == "groupby" and inner["table"] == "customer" and inner["keys"] == ["c_custkey"]
    assert d["columns"] == inner["columns"]  # the caller binds the body's tables
    step = inner["joins"][0]
    assert step["type"] == "left" and step["on"] == ["c_custkey", "o_custkey"]
    assert "o_comment" in step["on_filter"] and "special" in step["on_filter"]


def test_plan_grouped_derived_table():
    d = Plan("select m, count(*) as n from (select k, max(v) as m from t group by k) as d "
             "where m > 3 group by m").describe()
    assert d["table"] == "d" and d["derived"]["table"] == "t" and d["columns"] == ["k", "v"]
    assert d["where"] == [{"col": "m", "op": ">", "value": "3", "value_kind": "int"}]


def test_plan_on_filter_and_cte_errors():
    d = Plan("select count(*) from a join b on k = bk and w < 5").describe()
    assert d["joins"][0]["type"] == "inner" and "w" in d["joins"][0]["on_filter"]
    with pytest.raises(NutError, match="INNER, LEFT, SEMI and ANTI"):
        Plan("select count(*) from a right join b on k = bk and w < 5")
    with pytest.raises(NutError, match="needs an equality"):
        Plan("select count(*) from a join b on w < 5")
    with pytest.raises(NutError, match="WITH"):
        Plan("with c as (select k from t) select count(*) from u")
    with pytest.raises(NutError, match="not joined"):
        Plan("select count(*) from (select k, count(*) as c from t group by k) as d join u on d.k = u.k")
