"""CPU: the executor route of every single-table plan shape x {Int64, Float64} columns
(nut_plan_route — host only: binding, type checks and routing, nothing runs).

Row B1 (plan lowering): `Literal::Float` (/root/reference/src/parser/ast/
item.rs:89-101) and `ORDER BY` (/root/reference/src/parser/ast/query.rs:86-90) over Float64
columns.  Every FILTER / SORT / GROUPBY shape must route somewhere for both column types
(no "must be int64" rejection), and no Float64 ORDER BY key may reach an int64 sort on raw
bits: a single-key Float64 sort routes to `expr-sort-f64-order` (the bits mapped to the
IEEE total order before nut_sort_i64 and back after), and several keys / projections to the
row-id scan (nut_sort_pairs maps f64 keys itself).  GPU parity: tests/test_gpu_f64_scan.py.
"""
import itertools

import pytest

from nutdb_amd.sql import Plan

TYPES = ("int64", "float64")

SCANS = [
    "select x from t",
    "select x from t where x < 2",
    "select x from t where x < 1.5",
    "select x from t where x >= -3 and x <= 7",
    "select x from t where x between -1 and 1",
    "select x from t where x in (1, 2, 3)",
    "select x from t where x != 0",
    "select x from t where y < 10",
    "select x from t where x < 2 and y > 0",
    "select x, y from t",
    "select x, y from t where x > 0",
    "select x from t limit 10",
    "select x * 2 from t where x < 3",
    "select * from t where 1 = 1",
]
SORTS = [
    "select x from t order by x",
    "select x from t order by x desc",
    "select x from t order by x limit 100",
    "select x from t order by x desc limit 100",
    "select x from t order by x desc limit 100 offset 5",
    "select x from t where x < 2 order by x",
    "select x from t where x < 1.5 order by x desc limit 10",
    "select x from t where y < 3 order by x",
    "select y from t order by x",
    "select x, y from t order by x",
    "select x, y from t order by y desc, x",
    "select x from t order by y, x desc limit 7",
]
GROUPS = [
    "select y, sum(x) from t group by y",
    "select y, min(x), max(x), count(*) from t group by y",
    "select y, avg(x) from t where x < 2 group by y",
    "select sum(x), count(*) from t where x > 0",
    "select y, sum(x * 2) from t group by y",
    "select y, sum(x) from t group by y having sum(x) > 1 order by y desc limit 3",
    "select distinct y from t",
]


def route(sql, tx, ty):
    return Plan(sql).route({"x": tx, "y": ty})


@pytest.mark.parametrize("sql", SCANS + SORTS + GROUPS)
@pytest.mark.parametrize("tx,ty", list(itertools.product(TYPES, TYPES)))
def test_every_shape_routes(sql, tx, ty):
    r = route(sql, tx, ty)
    assert r, sql


@pytest.mark.parametrize("sql", SORTS)
@pytest.mark.parametrize("tx,ty", list(itertools.product(TYPES, TYPES)))
def test_no_float64_sort_on_raw_bits(sql, tx, ty):
    r = route(sql, tx, ty)
    final = r.split(" -> ")[-1]
    ordered = {"x": tx, "y": ty}[sql.split("order by")[1].split()[0].rstrip(",")]
    # single-key sorts hand int64 words to nut_sort_i64: raw bits only for int64 keys
    if final in ("fused-sort", "expr-sort"):
        assert ordered == "int64", (sql, r)
    elif final == "expr-sort-f64-order":
        assert ordered == "float64", (sql, r)
    else:
        assert final == "rowid-scan", (sql, r)


@pytest.mark.parametrize("sql,want", [
    ("select x from t", {"int64": "fused-filter", "float64": "rerun-expression -> expr-filter"}),
    ("select x from t where x < 2", {"int64": "fused-filter", "float64": "rerun-expression -> expr-filter"}),
    ("select x from t order by x", {"int64": "fused-sort", "float64": "rerun-expression -> expr-sort-f64-order"}),
    ("select x from t where x * 2 < 3 order by x desc limit 5",
     {"int64": "expr-sort", "float64": "expr-sort-f64-order"}),
    ("select x, y from t order by x", {"int64": "rowid-scan", "float64": "rowid-scan"}),
])
def test_route_names(sql, want):
    for t, r in want.items():
        assert route(sql, t, "int64") == r, (sql, t)


def test_float64_group_keys_route_to_key_words():
    """a Float64 GROUP BY column groups on int64 key words (IEEE total order, -0.0 = +0.0,
    one NaN) — fused, packed (> 2 keys) and DISTINCT alike"""
    assert route("select y, sum(x) from t group by y", "int64", "int64") == "fused-groupby"
    assert route("select y, sum(x) from t group by y", "int64", "float64") == "fused-groupby (float64 key words)"
    assert route("select x, y, count(*) from t group by x, y", "float64", "float64") == \
        "fused-groupby (float64 key words)"
    assert route("select distinct y from t", "int64", "float64").endswith("(float64 key words)")
    p = Plan("select x, y, x % 3 as z, count(*) from t group by x, y, z")
    assert p.route({"x": "int64", "y": "float64"}) == "packed-groupby (float64 key words)"


def test_computed_float64_group_key_is_a_plan_error():
    """a computed key of type float64 is refused by name (no grouping on raw bits)"""
    from nutdb_amd import NutError
    with pytest.raises(NutError, match="GROUP BY key 'y \\* 2' is float64"):
        route("select y * 2 as k, count(*) from t group by k", "int64", "float64")
