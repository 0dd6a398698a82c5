"""CPU: typed tables from CREATE TABLE (csrc/table.hip) — the schema
mapping of the reference's column types (src/parser/ast/item.rs:14-68) to executed HBM
columns, the rejected types, and string constants in plans (bound to dictionary codes
at execution, so they lower without a table)."""
import pytest

from nutdb_amd import NutError
from nutdb_amd.sql import Plan
from nutdb_amd.table import Table


def test_schema_mapping():
    t = Table(None, """CREATE TABLE lineitem (a Int8, b UInt16, c Float32, d Float64, e Boolean, f Date,
        g DateTime, h String, i Dictionary(String), j Enum('x' = 1, 'y' = 5), k Nullable(Int32), l Chars(4),
        m UInt64, n Int64, o Serial32, p USerial64)""")
    assert t.columns == {
        "a": (0, "int", 1), "b": (1, "uint", 2), "c": (2, "float", 4), "d": (3, "float", 8),
        "e": (4, "bool", 1), "f": (5, "date", 8), "g": (6, "datetime", 8), "h": (7, "string", 0),
        "i": (8, "string", 0), "j": (9, "enum", 8), "k": (10, "int", 4), "l": (11, "string", 0),
        "m": (12, "uint", 8), "n": (13, "int", 8), "o": (14, "int", 4), "p": (15, "uint", 8)}
    assert t.nrows == 0


@pytest.mark.parametrize("sql,status,frag", [
    ("CREATE TABLE t (a Int128)", "NUT_ERR_UNSUPPORTED", "128-bit"),
    ("CREATE TABLE t (a Decimal64(2))", "NUT_ERR_UNSUPPORTED", "Decimal"),
    ("CREATE TABLE t (a Uuid)", "NUT_ERR_UNSUPPORTED", "Uuid"),
    ("CREATE TABLE t (a Array(Int8))", "NUT_ERR_UNSUPPORTED", "Array"),
    ("CREATE TABLE t (a Map(String, Int8))", "NUT_ERR_UNSUPPORTED", "Map"),
    ("SELECT 1", "NUT_ERR_INVALID_ARG", "expected CREATE TABLE"),
    ("CREATE TABLE t (a Int8, a Int16)", "NUT_ERR_INVALID_ARG", "duplicate column"),
    ("CREATE TABLE t (a Int8", "NUT_ERR_PARSE", "Syntax Error"),
])
def test_schema_errors(sql, status, frag):
    with pytest.raises(NutError) as e:
        Table(None, sql)
    assert status in str(e.value) and frag in str(e.value)


def test_string_constants_lower():
    d = Plan("select l_shipmode, count(*) from t where l_shipmode in ('MAIL', 'SHIP') and x = 'a' "
             "group by l_shipmode").describe()
    assert d["mode"] == "fused"
    assert d["where"] == [{"col": "l_shipmode", "op": "in", "values": ["'MAIL'", "'SHIP'"]},
                          {"col": "x", "op": "=", "value": "'a'", "value_kind": "string"}]
    d = Plan("select k, sum(case when p = '1-URGENT' or p = '2-HIGH' then 1 else 0 end) from t "
             "where a = b or m = 'MAIL' group by k").describe()
    assert d["mode"] == "compiled" and d["where_expr"] == "((a = b) or (m = 'MAIL'))"
    assert d["aggs"][0]["expr"] == "if(((p = '1-URGENT') or (p = '2-HIGH')), 1, 0)"
    with pytest.raises(NutError) as e:
        Plan("select k, sum(v) from t group by k having k = 'a'")
    assert "string constants in HAVING" in str(e.value)
