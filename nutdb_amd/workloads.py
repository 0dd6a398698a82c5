"""Synthetic workloads of BASELINE.json configs 2-5.

Every column is a pure function of (seed, global row index) through the counter-based
splitmix64 generator, so any rank / shard / sample regenerates identical bits on the
device (nut_gen_column), in the C oracle (orc_gen_column) and in numpy
(tests/golden/make_golden.py).  Each entry: (name, nut_gen_kind, seed, a, b, c).
"""
from __future__ import annotations

from . import _lib as L

# config 2: SELECT col FROM t WHERE col < k     col uniform [0, 2^62)
FILTER_COL = ("col", L.GEN_U62, 0x2A, 0, 0, 1.0)


def filter_k(selectivity: float) -> int:
    return int(selectivity * 2**62)


# config 3: SELECT key, sum(val) ... GROUP BY key   key from a pool of G distinct i64
GB_KEY_SEED = 0x51
GB_VAL_SEED = 0x52


def groupby_cols(groups: int, dyadic: bool = True, skew: bool = False):
    """skew: Zipf-like keys from the same pool (GEN_SKEW_KEY: pool index i on ~1/i of the rows)."""
    return [
        ("key", L.GEN_SKEW_KEY if skew else L.GEN_POOL_KEY, GB_KEY_SEED, groups, 0, 1.0),
        ("val", L.GEN_DYADIC if dyadic else L.GEN_UNIT_F64, GB_VAL_SEED, 0, 0, 1.0),
    ]


# config 4: TPC-H Q1 shape (lineitem columns as i64 / f64)
Q1_DATE_K = 10471  # l_shipdate <= date '1998-12-01' - interval '90' day, as days since 1970
Q1_COLS = [
    ("l_shipdate", L.GEN_RANGE_I64, 0x41, 8036, 2526, 1.0),        # [8036, 10561]
    ("l_returnflag", L.GEN_RANGE_I64, 0x42, 0, 3, 1.0),             # {0,1,2} = A,N,R
    ("l_linestatus", L.GEN_RANGE_I64, 0x43, 0, 2, 1.0),             # {0,1}   = F,O
    ("l_quantity", L.GEN_RANGE_F64, 0x44, 1, 50, 1.0),              # 1..50
    ("l_extendedprice", L.GEN_RANGE_F64, 0x45, 90000, 10404901, 100.0),  # 900.00..104949.00
    ("l_discount", L.GEN_RANGE_F64, 0x46, 0, 11, 100.0),            # 0.00..0.10
]

# config 5: SELECT k FROM t ORDER BY k     full-range random i64
SORT_COL = ("k", L.GEN_FULL_I64, 0x50, 0, 0, 1.0)


def sort_col(key_range=None):
    """The sort column: full-range keys, or (key_range = f < 1/2) keys uniform over a
    fraction f of the int64 range — from 3 * 2^60 while it fits, else from -2^63 — the
    share one rank of an 8-GPU sample sort holds at f = 1/8."""
    if key_range is None:
        return SORT_COL
    width = int(float(key_range) * 2.0**64)
    assert 1 <= width <= 2**63 - 1, key_range
    start = 3 << 60 if width <= 5 << 60 else -(2**63)
    return ("k", L.GEN_RANGE_I64, 0x50, start, width, 1.0)

# Expression-mode workload: the reference fixture tests/sql/5.sql (TPC-H Q12 shape) with
# integer codes for its strings; 7 int64 columns = 56 B/row.
Q12_COLS = [
    ("o_orderkey", L.GEN_RANGE_I64, 0x61, 0, 4, 1.0),
    ("l_orderkey", L.GEN_RANGE_I64, 0x62, 0, 4, 1.0),
    ("l_shipmode", L.GEN_RANGE_I64, 0x63, 0, 7, 1.0),
    ("o_orderpriority", L.GEN_RANGE_I64, 0x64, 1, 5, 1.0),
    ("l_shipdate", L.GEN_RANGE_I64, 0x65, 8000, 2000, 1.0),
    ("l_commitdate", L.GEN_RANGE_I64, 0x66, 8000, 2000, 1.0),
    ("l_receiptdate", L.GEN_RANGE_I64, 0x67, 8000, 2000, 1.0),
]
Q12_SQL = """select l_shipmode,
    sum(case when o_orderpriority = 1 or o_orderpriority = 2 then 1 else 0 end) as high_line_count,
    sum(case when o_orderpriority <> 1 and o_orderpriority <> 2 then 1 else 0 end) as low_line_count
  from orders
  where o_orderkey = l_orderkey and l_shipmode in (3, 5) and l_commitdate < l_receiptdate
    and l_shipdate < l_commitdate
  group by l_shipmode
  order by l_shipmode"""
# the same query as the expression programs the planner lowers it to (column order
# = Q12_COLS), for the CPU baseline / oracle (oracle/expr.py)
_C = {name: i for i, (name, *_rest) in enumerate(Q12_COLS)}


def _col(n):
    return ("col", _C[n])


Q12_WHERE = [_col("o_orderkey"), _col("l_orderkey"), ("eq",), _col("l_shipmode"), ("i64", 0, 3), ("eq",),
             _col("l_shipmode"), ("i64", 0, 5), ("eq",), ("or",), ("and",), _col("l_commitdate"),
             _col("l_receiptdate"), ("lt",), ("and",), _col("l_shipdate"), _col("l_commitdate"), ("lt",), ("and",)]
Q12_AGGS = [
    (0, [_col("o_orderpriority"), ("i64", 0, 1), ("eq",), _col("o_orderpriority"), ("i64", 0, 2), ("eq",), ("or",),
         ("i64", 0, 1), ("i64", 0, 0), ("if",)], None),
    (0, [_col("o_orderpriority"), ("i64", 0, 1), ("ne",), _col("o_orderpriority"), ("i64", 0, 2), ("ne",), ("and",),
         ("i64", 0, 1), ("i64", 0, 0), ("if",)], None),
]


def gen(ex, spec, n: int, row0: int = 0):
    """Generate one column on ex's device."""
    _, kind, seed, a, b, c = spec
    return ex.gen_column(kind, seed, n, row0=row0, a=a, b=b, c=c)
