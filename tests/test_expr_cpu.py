"""CPU: expression mode (include/nutexec.h nut_prog; csrc/jit.cpp) without a GPU.

  * the numpy expression oracle (oracle/expr.py) against hand-computed answers for the
    edge cases the semantics define (wrap, truncating MOD/INTDIV, zero divisors, shifts,
    IF error scoping, int-vs-f64 compares);
  * nut_prog_type: result types and every malformed-program error;
  * SQL -> program lowering (describe): CASE/IF/multiIf, CASE without ELSE as an
    aggregate row mask, BETWEEN, IN beyond 16 values, column-vs-column comparisons;
  * the generated kernels compile with hipRTC for gfx950 (nut_plan_prepare), and the
    generated source does not depend on constants (one code object per query shape).
The expression semantics are this build's (the reference executes no expressions):
parity with the reference is unpinned for them; see oracle/expr.py.
"""
import ctypes as C

import numpy as np
import pytest

from nutdb_amd import _lib as L
from nutdb_amd import NutError, ProgQuery
from nutdb_amd.sql import Plan
from oracle.expr import BOOL, F64, I64, DivisionByZero, eval_prog, groupby_prog

I64MIN, I64MAX = -2**63, 2**63 - 1


def ev(nodes, *cols):
    v, t, e = eval_prog(nodes, [np.asarray(c) for c in cols])
    return v.tolist(), t, e.tolist()


def fbits(x):
    return int(np.array([x], dtype=np.float64).view(np.int64)[0])


# ------------------------------------------------------------------ oracle known answers
def test_oracle_integer_semantics():
    a = np.array([7, -7, 7, -7, I64MIN, I64MIN, 5], dtype=np.int64)
    b = np.array([2, 2, -2, -2, -1, 1, 0], dtype=np.int64)
    mod, t, err = ev([("col", 0), ("col", 1), ("mod",)], a, b)
    assert (mod, t) == ([1, -1, 1, -1, 0, 0, 0], I64) and err == [False] * 6 + [True]
    div, _, err = ev([("col", 0), ("col", 1), ("intdiv",)], a, b)
    assert div == [3, -3, -3, 3, I64MIN, I64MIN, 0] and err[-1]
    s, _, _ = ev([("col", 0), ("i64", 0, I64MAX), ("add",)], np.array([1], dtype=np.int64))
    assert s == [I64MIN]  # wraps
    m, _, _ = ev([("col", 0), ("col", 0), ("mul",)], np.array([2**32], dtype=np.int64))
    assert m == [0]
    ab, _, _ = ev([("col", 0), ("abs",)], np.array([I64MIN, -3], dtype=np.int64))
    assert ab == [I64MIN, 3]


def test_oracle_shifts_and_bits():
    x = np.array([1, -8, 1, -8, 3], dtype=np.int64)
    y = np.array([63, 1, 64, 70, -1], dtype=np.int64)
    assert ev([("col", 0), ("col", 1), ("shl",)], x, y)[0] == [I64MIN, -16, 0, 0, 0]
    assert ev([("col", 0), ("col", 1), ("shr",)], x, y)[0] == [0, -4, 0, -1, 0]
    assert ev([("col", 0), ("bitnot",)], x)[0] == [-2, 7, -2, 7, -4]
    assert ev([("col", 0), ("col", 1), ("bitxor",)], x, y)[0] == [62, -7, 65, -66, -4]


def test_oracle_compare_and_logic():
    i = np.array([2**53 + 1, 3, -1], dtype=np.int64)
    f = np.array([2.0**53, 3.0, float("nan")])
    v, t, _ = ev([("col", 0), ("col", 1), ("eq",)], i, f)
    assert t == BOOL and v == [1, 1, 0]  # the int converts to f64 (2^53+1 -> 2^53)
    assert ev([("col", 0), ("col", 1), ("ne",)], i, f)[0] == [0, 0, 1]  # NaN != x
    assert ev([("col", 0), ("i64", 0, 0), ("and",)], i)[0] == [0, 0, 0]
    assert ev([("col", 0), ("i64", 0, 0), ("or",)], i)[0] == [1, 1, 1]
    assert ev([("col", 0), ("not",)], np.array([0, 5], dtype=np.int64))[0] == [1, 0]
    assert ev([("col", 0), ("i64", 0, 1), ("div",)], np.array([7], dtype=np.int64))[1] == F64


def test_oracle_if_error_scope():
    a = np.array([10, 10, 10], dtype=np.int64)
    b = np.array([0, 5, 0], dtype=np.int64)
    # if(b != 0, a % b, -1): the MOD branch is not taken where b = 0 -> no error
    prog = [("col", 1), ("i64", 0, 0), ("ne",), ("col", 0), ("col", 1), ("mod",), ("i64", 0, -1), ("if",)]
    v, t, err = ev(prog, a, b)
    assert v == [-1, 0, -1] and err == [False, False, False]
    # AND evaluates both operands: (b != 0) and (a % b = 0) raises where b = 0
    prog = [("col", 1), ("i64", 0, 0), ("ne",), ("col", 0), ("col", 1), ("mod",), ("i64", 0, 0), ("eq",), ("and",)]
    assert ev(prog, a, b)[2] == [True, False, True]


def test_oracle_groupby_error_rule():
    k = np.array([1, 1, 2], dtype=np.int64)
    a = np.array([6, 7, 8], dtype=np.int64)
    b = np.array([0, 2, 0], dtype=np.int64)
    where = [("col", 1), ("i64", 0, 0), ("ne",)]
    val = [("col", 0), ("col", 1), ("mod",)]
    keys, words, types = groupby_prog([k], [a, b], where, [(0, val, None), (1, None, None)])
    assert keys.tolist() == [[1]] and words.tolist() == [[1, 1]] and types == [I64, I64]
    with pytest.raises(DivisionByZero):
        groupby_prog([k], [a, b], None, [(0, val, None)])
    # masked-out rows do not raise either
    mask = [("col", 1), ("i64", 0, 0), ("gt",)]
    keys, words, _ = groupby_prog([k], [a, b], None, [(0, val, mask), (1, None, mask)])
    assert keys.tolist() == [[1], [2]] and words.tolist() == [[1, 1], [0, 0]]


# ------------------------------------------------------------------ nut_prog_type
def prog_type(nodes, col_types):
    keep = []
    from nutdb_amd.executor import _prog
    pr = _prog(nodes, keep)
    ct = (C.c_int32 * max(len(col_types), 1))(*col_types)
    t = C.c_int32()
    st = L.lib.nut_prog_type(C.byref(pr), ct, len(col_types), C.byref(t))
    if st:
        raise NutError(st, "nut_prog_type", L.lib.nut_last_error().decode())
    return t.value


def test_prog_types():
    I, F = L.T_I64, L.T_F64
    assert prog_type([("col", 0), ("col", 1), ("add",)], [I, I]) == L.PT_I64
    assert prog_type([("col", 0), ("col", 1), ("add",)], [I, F]) == L.PT_F64
    assert prog_type([("col", 0), ("col", 1), ("div",)], [I, I]) == L.PT_F64
    assert prog_type([("col", 0), ("col", 1), ("lt",)], [I, F]) == L.PT_BOOL
    assert prog_type([("col", 0), ("i64", 0, 1), ("f64", 0, 2.5), ("if",)], [I]) == L.PT_F64
    assert prog_type([("col", 0), ("i64", 0, 1), ("i64", 0, 2), ("if",)], [I]) == L.PT_I64
    assert prog_type([("col", 0), ("to_f64",)], [I]) == L.PT_F64


@pytest.mark.parametrize("nodes,types,frag", [
    ([], [], "empty"),
    ([("add",)], [], "underflow"),
    ([("col", 3)], [0], "out of range"),
    ([("col", 0), ("col", 0)], [0], "leaves 2"),
    ([("col", 0), ("col", 0), ("bitand",)], [1], "integer operands"),
    ([("col", 0), ("col", 0), ("intdiv",)], [1], "integer operands"),
    ([("col", 0), ("not",)], [1], "float64"),
    ([("col", 0), ("col", 0), ("col", 0), ("if",)], [1], "IF condition"),
    ([(99, 0, 0)], [0], "unknown program op"),
])
def test_prog_type_errors(nodes, types, frag):
    with pytest.raises(NutError) as e:
        prog_type(nodes, types)
    assert frag in str(e.value)


def test_prog_too_long():
    with pytest.raises(ValueError):
        ProgQuery(keys=[], cols=[], aggs=[], where=[("i64", 0, 1)] * 300).to_spec(None)


# ------------------------------------------------------------------ SQL lowering
def test_plan_compiled_q12_shape():
    # tests/golden/sql/5.sql (the reference's fixture) with integer codes for the strings
    d = Plan("""select l_shipmode,
        sum(case when o_orderpriority = 1 or o_orderpriority = 2 then 1 else 0 end) as high_line_count,
        sum(case when o_orderpriority <> 1 and o_orderpriority <> 2 then 1 else 0 end) as low_line_count
      from orders
      where o_orderkey = l_orderkey and l_shipmode in (3, 5) and l_commitdate < l_receiptdate
        and l_shipdate < l_commitdate
      group by l_shipmode order by l_shipmode""").describe()
    assert d["mode"] == "compiled" and d["kind"] == "groupby"
    assert d["where_expr"] == ("((((o_orderkey = l_orderkey) and ((l_shipmode = 3) or (l_shipmode = 5))) and "
                               "(l_commitdate < l_receiptdate)) and (l_shipdate < l_commitdate))")
    assert d["aggs"] == [
        {"op": "sum", "expr": "if(((o_orderpriority = 1) or (o_orderpriority = 2)), 1, 0)"},
        {"op": "sum", "expr": "if(((o_orderpriority != 1) and (o_orderpriority != 2)), 1, 0)"}]
    assert [o["name"] for o in d["outputs"]] == ["l_shipmode", "high_line_count", "low_line_count"]


def test_plan_null_branches_become_masks():
    d = Plan("select k, sum(case when v > 0 then v end), avg(case when v > 0 then v end), "
             "count(case when v > 0 then 1 end), count(v), min(case v when 1 then w when 2 then null else 0 end) "
             "from t group by k").describe()
    aggs = d["aggs"]
    assert aggs[0] == {"op": "sum", "expr": "if((v > 0), v, 0)", "mask": "if((v > 0), true, false)"}
    # avg = the same sum + a count under the same mask (shared with count(case ...));
    # count(v) has no mask
    out = d["outputs"][2]
    assert (out["from"], out["sum"], out["count"]) == ("avg", 0, 1)
    assert aggs[1] == {"op": "count", "mask": aggs[0]["mask"]}
    assert d["outputs"][3]["index"] == 1 and {"op": "count"} in aggs
    assert aggs[-1]["op"] == "min" and aggs[-1]["mask"] == "if((v = 1), true, if((v = 2), false, true))"


def test_plan_fused_stays_fused():
    d = Plan("select k, sum(v), count(*) from t where k < 5 and v >= 0.5 group by k").describe()
    assert d["mode"] == "fused"
    d = Plan("select k, sum(v) from t where k < 5 or v >= 0.5 group by k").describe()
    assert d["mode"] == "compiled" and d["where_expr"] == "((k < 5) or (v >= 0.5))"
    d = Plan("select sum(a * b * c), max(intDiv(a, 3)), min(a % 4) from t where a between 1 and 9").describe()
    assert d["mode"] == "compiled" and d["keys"] == []
    assert [a.get("expr") for a in d["aggs"]] == ["((a * b) * c)", "(a div 3)", "(a % 4)"]
    assert d["where_expr"] == "((a >= 1) and (a <= 9))"


def test_plan_scan_modes():
    """one comparison of the projected column stays on the filter kernel; any other WHERE
    makes an expression-mode scan (nut_select_rows), ORDER BY / LIMIT included"""
    assert Plan("select x from t where x < 5").describe()["mode"] == "fused"
    for sql, where in [("select x from t where x < y", "(x < y)"),
                       ("select x from t where x > 1 and x < 9", "((x > 1) and (x < 9))"),
                       ("select x from t where y in (1, 2)", "((y = 1) or (y = 2))"),
                       ("select x from t where x % 3 = 0 order by x desc limit 4", "((x % 3) = 0)")]:
        d = Plan(sql).describe()
        assert d["mode"] == "compiled" and d["where_expr"] == where, sql
    assert Plan("select x from t where x % 3 = 0 order by x desc limit 4").kind == "sort"


@pytest.mark.parametrize("sql,types", [
    ("select x from t where x < y", {"x": "int64", "y": "int64"}),
    ("select x from t where y * 2.5 > 1 or not (x between 3 and 8) order by x", {"x": "int64", "y": "float64"}),
    ("select x from t where multiIf(x = 1, y, x = 2, 2 * y, 0) > 0.5", {"x": "int64", "y": "float64"})])
def test_scan_jit_compiles(sql, types):
    """the scan kernel (select_kernel.hpp) of expression-mode scans compiles with hipRTC"""
    Plan(sql).prepare(types)


# ------------------------------------------------------------------ hipRTC
COMPILE_CASES = [
    ("select k, sum(a + b), sum(a - b), sum(a * b), max(a / b), min(a % b), max(intDiv(a, b)) from t group by k",
     {"a": "int64", "b": "int64"}),
    ("select k, count(*), min(a & b), max(a | b), sum(a ^ b), sum(a << 3), sum(b >> 2), max(~a) from t "
     "where not (a < b) and (a > 0 xor b > 0) group by k", {"a": "int64", "b": "int64"}),
    ("select k, j, sum(case when x < 0.5 then x when x < 0.75 then 2 * x else abs(x) end), "
     "avg(case when y > 0 then y end), max(toFloat64(y)) from t where x between 0.1 and 0.9 or y in (1, 2, 3) "
     "group by k, j", {"x": "float64", "y": "int64"}),
    ("select sum(multiIf(a = 1, b, a = 2, 2 * b, 0)), count(case a when 1 then 1 when 2 then 1 end) from t "
     "where a is not null", {"a": "int64", "b": "float64"}),
]


@pytest.mark.parametrize("sql,types", COMPILE_CASES)
def test_jit_compiles(sql, types):
    p = Plan(sql)
    assert p.describe()["mode"] == "compiled"
    p.prepare({**types, "k": "int64", "j": "int64"})


def test_jit_type_error_is_a_plan_error():
    p = Plan("select k, sum(x & 1) from t group by k")
    with pytest.raises(NutError) as e:
        p.prepare({"k": "int64", "x": "float64"})
    assert "NUT_ERR_PLAN" in str(e.value) and "integer operands" in str(e.value)


def jit_source(q):
    spec = q.to_spec(None)
    buf = C.create_string_buffer(1 << 16)
    n = C.c_size_t()
    st = L.lib.nut_groupby_jit_source(C.byref(spec), buf, len(buf), C.byref(n))
    assert st == 0, L.lib.nut_last_error()
    return buf.value.decode()


class _FakeCol:
    """stands in for a tensor when only types matter (no device pointer is read)"""

    def __init__(self, dtype):
        import torch
        self.dtype = dtype
        self.device = None
        self._t = torch.empty(0, dtype=dtype)

    def numel(self):
        return 0

    def is_contiguous(self):
        return True

    def dim(self):
        return 1

    def data_ptr(self):
        return 0


def test_jit_source_independent_of_constants():
    import torch
    cols = [_FakeCol(torch.int64), _FakeCol(torch.float64)]
    mk = lambda c, f: ProgQuery(keys=[], cols=cols, where=[("col", 0), ("i64", 0, c), ("lt",)],
                                aggs=[("sum", [("col", 1), ("f64", 0, f), ("mul",)], None)])
    s1, s2 = jit_source(mk(5, 2.5)), jit_source(mk(-123, 0.125))
    assert s1 == s2 and "p.kc[0]" in s1 and "p.kc[1]" in s1
    assert "5" not in s1.split("where")[1].split(";")[0].replace("p.kc", "")


def test_plan_scan_several_columns():
    d = Plan("select a, b as bb, c from t where a > 1 or c < 0").describe()
    assert d["kind"] == "filter" and d["mode"] == "compiled" and d["project"] == ["a", "b", "c"]
    assert [o["name"] for o in d["outputs"]] == ["a", "bb", "c"]
    # ORDER BY with projected columns: row ids sorted by the keys, columns gathered
    d = Plan("select a, b from t where a > 1 order by a").describe()
    assert d["kind"] == "sort" and d["mode"] == "compiled" and d["sort"] == [{"column": "a", "desc": False}]
    d = Plan("select a, b as bb from t order by bb desc, z").describe()
    assert d["sort"] == [{"column": "b", "desc": True}, {"column": "z", "desc": False}]
    assert d["project"] == ["a", "b"] and "z" in d["columns"]
    with pytest.raises(NutError, match="is not a column"):
        Plan("select a from t order by a + 1")


def test_plan_select_distinct():
    d = Plan("select distinct k, j from t where x > 3 order by k desc limit 5").describe()
    assert d["kind"] == "groupby" and d["keys"] == ["k", "j"] and d["aggs"] == [{"op": "count"}]
    assert [o["name"] for o in d["outputs"]] == ["k", "j"]
    d = Plan("select distinct a, b, c from t").describe()
    assert d["mode"] == "compiled" and d["keys"] == ["a", "b", "c"]
    for sql, msg in [("select distinct count(*) from t", "over aggregates"),
                     ("select distinct k from t group by k", "with GROUP BY"),
                     ("select distinct a, b, c, d, e, f, g, h, i from t", "1 to 8 columns")]:
        with pytest.raises(NutError, match=msg):
            Plan(sql)


def test_plan_like():
    d = Plan("select count(*) from t where s like 'AB%' and not (s ilike '%x_')").describe()
    assert d["mode"] == "compiled" and d["where_expr"] == "((s like 'AB%') and not((s ilike '%x_')))"
    assert Plan("select s from t where s not like '%Z'").describe()["where_expr"] == "not((s like '%Z'))"
    with pytest.raises(NutError, match="string pattern"):
        Plan("select count(*) from t where s like 3")


# ------------------------------------------------------------------ GROUP BY keys (§3.6)
def test_plan_many_and_computed_keys():
    d = Plan("select a, b, c, count(*) from t group by a, b, c").describe()
    assert d["mode"] == "compiled" and d["keys"] == ["a", "b", "c"]
    assert [o["from"] for o in d["outputs"]] == ["key", "key", "key", "agg"]
    # a SELECT alias names its expression; getYear is ClickHouse's toYear
    d = Plan("select getYear(d) as y, sum(v) from t group by y order by y").describe()
    assert d["keys"] == ["getYear(d)"] and d["outputs"][0] == {"name": "y", "from": "key", "index": 0}
    d = Plan("select toMonth(d), a % 10 as r, count() from t group by toMonth(d), r").describe()
    assert d["keys"] == ["toMonth(d)", "a % 10"] and [o["from"] for o in d["outputs"]] == ["key", "key", "agg"]
    # date functions of constants fold
    d = Plan("select count() from t where getYear(d) = getYear(toDate('1996-03-01')) "
             "and toDayOfWeek(d) < toDayOfWeek(toDate('2024-06-09'))").describe()
    assert d["where_expr"] == "((toYear(d) = 1996) and (toDayOfWeek(d) < 7))"
    with pytest.raises(NutError, match="1 to 8 keys"):
        Plan("select count() from t group by a, b, c, d, e, f, g, h, i")
    with pytest.raises(NutError, match="neither a GROUP BY key"):
        Plan("select a, b, count() from t group by a, c, d")


def test_plan_count_unique_and_output_arithmetic():
    d = Plan("select k, countUnique(x) as u, uniqExact(x), sum(v) / count() as m, 100.0 * sum(v) / sum(w) "
             "from t group by k having sum(v) - sum(w) > 3 order by m desc").describe()
    assert d["aggs"][0] == {"op": "count_distinct", "expr": "x"}
    assert [o["from"] for o in d["outputs"] if not o.get("hidden")] == ["key", "agg", "agg", "expr", "expr"]
    assert d["outputs"][2]["index"] == d["outputs"][1]["index"]  # uniqExact(x) = countUnique(x)
    d = Plan("select countUnique(case when v > 0 then x end) from t").describe()
    assert d["keys"] == [] and d["aggs"][0]["op"] == "count_distinct" and "mask" in d["aggs"][0]
    for sql, msg in [("select k, sum(v) > 3 from t group by k", "not executed over aggregates"),
                     ("select k, v + sum(v) from t group by k", "not a GROUP BY key, an aggregate"),
                     ("select k, countUnique(x, y) from t group by k", "takes one argument")]:
        with pytest.raises(NutError, match=msg):
            Plan(sql)


def test_jit_compiles_key_programs():
    """computed keys (nut_agg_spec.key_prog) compile into the streaming kernel (hipRTC)"""
    import torch
    cols = [_FakeCol(torch.int64), _FakeCol(torch.float64)]
    yr = [("col", 0), ("datepart", L.DP_YEAR), ("i64", 0, 1970), ("sub",), ("i64", 0, 40), ("shl",),
          ("col", 0), ("datepart", L.DP_MONTH), ("bitor",)]
    q = ProgQuery(keys=[yr, [("col", 0), ("i64", 0, 7), ("mod",)]], cols=cols,
                  aggs=[("sum", [("col", 1)], None), ("count", None, None)])
    src = jit_source(q)
    assert "kKeyProg = 3" in src and "jdatepart(" in src
    assert L.lib.nut_groupby_jit_compile(C.byref(q.to_spec(None))) == 0, L.lib.nut_last_error()
    bad = ProgQuery(keys=[[("col", 1)]], cols=cols, aggs=[("count", None, None)])
    assert L.lib.nut_groupby_jit_compile(C.byref(bad.to_spec(None))) != 0
    assert b"float64" in L.lib.nut_last_error()


def test_date_part_oracle_matches_calendar():
    """oracle.expr.date_part (the DATEPART restatement) against Python's proleptic
    Gregorian calendar, years 1 .. 9999"""
    import datetime
    from oracle.expr import date_part
    rng = np.random.default_rng(3)
    lo, hi = datetime.date(1, 1, 1).toordinal(), datetime.date(9999, 12, 31).toordinal()
    epoch = datetime.date(1970, 1, 1).toordinal()
    ords = np.concatenate([rng.integers(lo, hi + 1, 20000), np.arange(epoch - 800, epoch + 800),
                           [lo, hi, datetime.date(2000, 2, 29).toordinal(), datetime.date(1900, 3, 1).toordinal()]])
    days = (ords - epoch).astype(np.int64)
    dates = [datetime.date.fromordinal(int(o)) for o in ords]
    want = {
        0: [x.year for x in dates], 1: [x.month for x in dates], 2: [x.day for x in dates],
        3: [(x.month - 1) // 3 + 1 for x in dates], 4: [x.isoweekday() for x in dates],
        5: [x.timetuple().tm_yday for x in dates],
        6: [x.year * 100 + x.month for x in dates], 7: [int(x.strftime("%Y%m%d")) for x in dates],
    }
    for part, w in want.items():
        assert date_part(days, part).tolist() == w, part
    # beyond any date the input is clamped to +-2^40 days
    big = np.array([2**62, -2**62, 2**40, -2**40], dtype=np.int64)
    assert date_part(big, 0).tolist() == [date_part(np.array([2**40]), 0)[0]] * 1 + \
        [date_part(np.array([-2**40]), 0)[0]] + date_part(big[2:], 0).tolist()


def test_plan_computed_projections():
    """SELECT items that are expressions (no aggregate anywhere) are computed projections of
    an expression-mode scan (nut_eval_rows on the selected rows); a CASE without ELSE is a
    NULL mask; an aggregate inside arithmetic makes a global aggregate instead."""
    d = Plan("select a * 2 + b as s, toYYYYMMDD(d), a from t where a > 1 order by a limit 3").describe()
    assert d["kind"] == "sort" and d["mode"] == "compiled"
    assert d["project"] == ["((a * 2) + b)", "toYYYYMMDD(d)", "a"]
    assert [o["name"] for o in d["outputs"]] == ["s", "toYYYYMMDD(d)", "a"]
    d = Plan("select abs(x), case when x > 0 then x end from t").describe()
    assert d["kind"] == "filter" and d["mode"] == "compiled" and len(d["project"]) == 2
    assert Plan("select sum(a) / sum(b) from t").kind == "groupby"
    with pytest.raises(NutError, match="ORDER BY a computed projection"):
        Plan("select a + 1 as c from t order by c")


@pytest.mark.parametrize("sql,types", [
    ("select a * 2 + b, toYYYYMM(d), case when b > 0.5 then b end from t where a > 1",
     {"a": "int64", "b": "float64", "d": "int64"}),
    ("select " + ", ".join(f"a + {i}" for i in range(10)) + " from t order by a",
     {"a": "int64"})])
def test_eval_jit_compiles(sql, types):
    """the evaluation kernels (select_kernel.hpp eval_kernel, <= 8 programs each) of computed
    projections compile with hipRTC next to the scan kernel"""
    Plan(sql).prepare(types)


def test_plan_select_star():
    """SELECT * (the reference's criterion statement `SELECT * FROM table WHERE 1 = 1`,
    benches/parser.rs): every column bound at execution, in binding order"""
    d = Plan("SELECT * FROM table WHERE 1 = 1").describe()
    assert d["kind"] == "filter" and d["column"] == "*" and d["mode"] == "compiled" and d["where_expr"] == ""
    d = Plan("select * from t where a > 3 order by b desc limit 2").describe()
    assert d["kind"] == "sort" and d["sort"] == [{"column": "b", "desc": True}] and d["limit"] == 2
    for sql, frag in [("select *, a from t", "alone"), ("select t.* from t", "unqualified"),
                      ("select * from a join b on x = y", "over a JOIN")]:
        with pytest.raises(NutError, match=frag):
            Plan(sql)
    Plan("select * from t where a > 1.5 and b < 3").prepare({"a": "int64", "b": "float64", "c": "int64"})


def test_c_integer_evaluator_matches_numpy_oracle():
    """oracle.eval_int (the CPU baseline's C evaluator of integer / bool programs) equals
    eval_prog on random programs of its subset over columns with extremes, and declines
    programs outside it (f64, MOD, shifts)."""
    from oracle import oracle as orc
    rng = np.random.default_rng(7)
    n = (1 << 20) + 77
    cols = [rng.integers(-5, 6, n), rng.integers(I64MIN, I64MAX, n, endpoint=True), rng.integers(0, 3, n)]
    cols[1][:4] = [I64MIN, I64MAX, 0, -1]
    bin_ops = ["add", "sub", "mul", "lt", "le", "gt", "ge", "eq", "ne", "and", "or", "xor", "bitand", "bitor",
               "bitxor"]
    for trial in range(40):
        prog, depth = [], 0
        for _ in range(int(rng.integers(1, 14))):
            r = rng.random()
            if depth >= 3 and r < 0.2:
                prog.append(("if",))
                depth -= 2
            elif depth >= 2 and r < 0.7:
                prog.append((bin_ops[int(rng.integers(len(bin_ops)))],))
                depth -= 1
            elif depth >= 1 and r < 0.78:
                prog.append((["not", "bitnot"][int(rng.integers(2))],))
            elif r < 0.9:
                prog.append(("col", int(rng.integers(3))))
                depth += 1
            else:
                prog.append(("i64", 0, int(rng.integers(-9, 10))))
                depth += 1
        while depth > 1:
            prog.append(("add",))
            depth -= 1
        if depth == 0:
            prog = [("col", 1)]
        want, _, err = eval_prog(prog, cols)
        got = orc.eval_int(prog, cols, n)
        assert got is not None, prog
        assert not err.any() and np.array_equal(got, want), (trial, prog)
    assert orc.eval_int([("col", 0), ("col", 1), ("mod",)], cols, n) is None
    assert orc.eval_int([("col", 0), ("i64", 0, 3), ("shl",)], cols, n) is None
    assert orc.eval_int([("col", 0)], [np.zeros(n)], n) is None
