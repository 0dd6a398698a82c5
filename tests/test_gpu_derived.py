"""Grouped derived tables, CTEs and JOIN ON filters on the GPU, against
pandas.

The reference's fixture tests/sql/6.sql is TPC-H Q13's shape: a CTE
`c_orders AS (SELECT c_custkey, count(o_orderkey) AS c_count FROM customer LEFT OUTER JOIN
orders ON c_custkey = o_custkey AND o_comment NOT LIKE '%special%requests%' GROUP BY
c_custkey)` read by an outer GROUP BY over its output.  The executor materializes the grouped
body (nut_plan::inner) and runs the outer plan over its result columns; the ON filter on
the JOIN source (`o_comment NOT LIKE ..`) filters `orders` before the LEFT join (so a
customer whose orders all fail it still counts, with 0).  The fixture's own outer WHERE
compares `total_revenue` with a subquery over `revenue0`, a table the query never defines,
so Q13 runs here without that conjunct.  Counts and keys bit-exact."""
import numpy as np
import pandas as pd
import pytest
import torch

from nutdb_amd.table import Table

pytestmark = pytest.mark.gpu

Q13 = """with c_orders as (
    select c_custkey, count(o_orderkey) as c_count
    from customer left outer join orders on c_custkey = o_custkey
        and o_comment not like '%special%requests%'
    group by c_custkey
)
select c_count, count(*) as custdist
from c_orders
group by c_count
order by custdist desc, c_count desc"""


def on_dev(ex, cols):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(ex.device) for k, v in cols.items()}


def q13_oracle(cust, orders, keep):
    o = pd.DataFrame(orders)[keep]
    per = o.groupby("o_custkey").size()
    cnt = pd.Series(cust["c_custkey"]).map(per).fillna(0).astype(np.int64)
    g = cnt.value_counts().reset_index()
    g.columns = ["c_count", "custdist"]
    return g.sort_values(["custdist", "c_count"], ascending=[False, False])


def test_q13_cte_left_join_on_filter_typed_tables(ex):
    rng = np.random.default_rng(13)
    nc, no = 30_000, 300_000
    ck = rng.permutation(nc * 2)[:nc].astype(np.int64)
    words = np.array(["special", "requests", "pending", "deposits", "quickly", "final"], dtype=object)
    comments = np.array([" ".join(rng.choice(words, 3)) for _ in range(no)], dtype=object)
    orders = {"o_orderkey": np.arange(no, dtype=np.int64),
              "o_custkey": np.where(rng.random(no) < 0.7, rng.choice(ck, no), rng.integers(nc * 2, nc * 3, no)).astype(np.int64),
              "o_comment": comments}
    cust = {"c_custkey": ck}
    tc = Table(ex, "CREATE TABLE customer (c_custkey Int64)")
    tc.append(**cust)
    to = Table(ex, "CREATE TABLE orders (o_orderkey Int64, o_custkey Int64, o_comment String)")
    to.append(**orders)
    got = tc.sql(Q13, right=to)
    keep = ~pd.Series(comments).str.contains("special.*requests", regex=True).to_numpy()
    assert 0.1 < keep.mean() < 0.95
    want = q13_oracle(cust, orders, keep)
    assert got["c_count"].tolist() == want.c_count.tolist()
    assert got["custdist"].tolist() == want.custdist.tolist()
    assert sum(got["custdist"]) == nc and 0 in got["c_count"].tolist()


def test_grouped_derived_table_and_on_filter_raw_columns(ex):
    """FROM (SELECT .. GROUP BY ..) AS d with an outer WHERE on its output and an outer
    GROUP BY; a LEFT JOIN whose ON filters the JOIN source numerically."""
    rng = np.random.default_rng(14)
    nc, no = 20_000, 200_000
    ck = np.arange(nc, dtype=np.int64)
    orders = {"o_custkey": rng.integers(0, nc + 500, no).astype(np.int64),
              "o_price": rng.integers(1, 1000, no).astype(np.int64),
              "o_orderkey": np.arange(no, dtype=np.int64)}
    q = ("select c_count, count(*) as custdist, sum(big) as big_total from "
         "(select c_custkey, count(o_orderkey) as c_count, max(o_price) as big from customer left join orders "
         "on c_custkey = o_custkey and o_price > 500 group by c_custkey) as d "
         "where c_count > 0 group by c_count order by c_count")
    got = ex.sql(q, on_dev(ex, {"c_custkey": ck}), right=on_dev(ex, orders))
    do = pd.DataFrame(orders)
    o = do[do.o_price > 500]
    inner = pd.DataFrame({"c_custkey": ck}).merge(o, left_on="c_custkey", right_on="o_custkey", how="left")
    per = inner.groupby("c_custkey").agg(c_count=("o_orderkey", "count"), big=("o_price", "max")).reset_index()
    per = per[per.c_count > 0]
    want = per.groupby("c_count").agg(custdist=("c_custkey", "size"), big_total=("big", "sum")).reset_index()
    assert got["c_count"].tolist() == want.c_count.tolist()
    assert got["custdist"].tolist() == want.custdist.tolist()
    assert np.array_equal(np.asarray(got["big_total"], dtype=np.int64), want.big_total.to_numpy(np.int64))


def test_inner_join_on_filter_and_single_table_derived(ex):
    rng = np.random.default_rng(15)
    n = 100_000
    a = {"k": rng.integers(0, 5000, n).astype(np.int64), "v": rng.integers(0, 100, n).astype(np.int64)}
    b = {"bk": np.arange(5000, dtype=np.int64), "w": rng.integers(0, 10, 5000).astype(np.int64)}
    got = ex.sql("select w, count(*) as c from a join b on k = bk and w < 5 group by w order by w",
                 on_dev(ex, a), right=on_dev(ex, b))
    da, db = pd.DataFrame(a), pd.DataFrame(b)
    m = da.merge(db[db.w < 5], left_on="k", right_on="bk")
    want = m.groupby("w").size()
    assert got["w"].tolist() == want.index.tolist() and got["c"].tolist() == want.tolist()
    # a grouped derived table over one table, its outputs renamed and filtered
    got = ex.sql("select mx, count(*) as n from (select k, max(v) as mx from a group by k) as t "
                 "where mx >= 90 group by mx order by mx", on_dev(ex, a))
    per = da.groupby("k").v.max()
    want = per[per >= 90].value_counts().sort_index()
    assert got["mx"].tolist() == want.index.tolist() and got["n"].tolist() == want.tolist()
