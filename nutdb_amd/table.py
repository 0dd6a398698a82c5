"""Typed device tables from CREATE TABLE (csrc/table.hip).

    t = Table(ex, "CREATE TABLE lineitem (l_returnflag String, l_quantity Int8, ...)")
    t.append(l_returnflag=["A", "N", ...], l_quantity=np.array([...], np.int8), ...)
    t.sql("SELECT l_returnflag, sum(l_quantity) FROM lineitem GROUP BY l_returnflag")

Columns live in HBM in the executed representation (int64 / f64); narrow integers and
Float32 cross PCIe at their declared width and are widened on the GPU; strings are
dictionary-encoded (codes feed the same int64 kernels; string constants in a query bind
to codes; string group keys come back as str).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List

import numpy as np

from . import _lib as L
from ._lib import check, lib
from .sql import Plan, read_result

# numpy dtype a numeric column takes, per (kind, width)
_NP = {("int", 1): np.int8, ("int", 2): np.int16, ("int", 4): np.int32, ("int", 8): np.int64,
       ("uint", 1): np.uint8, ("uint", 2): np.uint16, ("uint", 4): np.uint32, ("uint", 8): np.uint64,
       ("float", 4): np.float32, ("float", 8): np.float64, ("bool", 1): np.uint8,
       ("date", 8): np.int64, ("datetime", 8): np.int64}


class Table:
    def __init__(self, ex, create_sql: str):
        self.ex = ex
        b = create_sql.encode("utf-8")
        h = C.c_void_p()
        check(lib.nut_table_create(b, len(b), C.byref(h)), "nut_table_create")
        self._h = h
        nc = C.c_int()
        check(lib.nut_table_shape(h, C.byref(nc), None), "nut_table_shape")
        self.columns = {}
        for j in range(nc.value):
            nm, kind, width, et = C.c_char_p(), C.c_int(), C.c_int(), C.c_int()
            check(lib.nut_table_column_info(h, j, C.byref(nm), C.byref(kind), C.byref(width), C.byref(et)),
                  "nut_table_column_info")
            self.columns[nm.value.decode()] = (j, L.COL_KINDS[kind.value], width.value)

    @property
    def nrows(self) -> int:
        n = C.c_uint64()
        check(lib.nut_table_shape(self._h, None, C.byref(n)), "nut_table_shape")
        return n.value

    def append(self, **cols) -> None:
        """Append values column by column (host data); every column must end up with the
        same number of rows before a query runs."""
        self.ex._bind_stream()
        for name, values in cols.items():
            if name not in self.columns:
                raise KeyError(f"no column {name!r}")
            j, kind, width = self.columns[name]
            if kind in ("string", "enum"):
                enc = [str(v).encode("utf-8") for v in values]
                off = np.zeros(len(enc) + 1, dtype=np.int64)
                np.cumsum([len(x) for x in enc], out=off[1:])
                data = b"".join(enc)
                buf = C.create_string_buffer(data, len(data) + 1)
                check(lib.nut_table_append(self.ex.ctx, self._h, j, buf, off.ctypes.data_as(C.c_void_p), len(enc)),
                      "nut_table_append")
            else:
                if kind == "date" and len(values) and isinstance(values[0], str):
                    values = (np.array(values, dtype="datetime64[D]") - np.datetime64("1970-01-01", "D")).astype(np.int64)
                a = np.ascontiguousarray(values, dtype=_NP[(kind, width)])
                check(lib.nut_table_append(self.ex.ctx, self._h, j, a.ctypes.data_as(C.c_void_p), None, len(a)),
                      "nut_table_append")

    def execute(self, plan: Plan, group_hint: int = 0) -> Dict[str, np.ndarray]:
        res = C.c_void_p()
        self.ex._bind_stream()
        check(lib.nut_table_execute(self.ex.ctx, self._h, plan._handle(), group_hint, C.byref(res)),
              "nut_table_execute")
        return read_result(res)

    def execute_join(self, plan: Plan, right: "Table", group_hint: int = 0) -> Dict[str, np.ndarray]:
        """A JOIN plan with this table as the FROM side and `right` as the JOIN source
        (nut_table_execute2): string columns carry their own dictionaries through the join."""
        res = C.c_void_p()
        self.ex._bind_stream()
        check(lib.nut_table_execute2(self.ex.ctx, self._h, right._h, plan._handle(), group_hint, C.byref(res)),
              "nut_table_execute2")
        return read_result(res)

    def execute_joins(self, plan: Plan, joined: List["Table"], group_hint: int = 0) -> Dict[str, np.ndarray]:
        """A chain of JOINs with this table as FROM and `joined[k]` as the k-th JOIN source
        (nut_table_executen), strings as in execute_join."""
        res = C.c_void_p()
        self.ex._bind_stream()
        hs = (C.c_void_p * (len(joined) + 1))(self._h, *[t._h for t in joined])
        check(lib.nut_table_executen(self.ex.ctx, hs, len(joined) + 1, plan._handle(), group_hint, C.byref(res)),
              "nut_table_executen")
        return read_result(res)

    def sql(self, query: str, group_hint: int = 0, right: "Table" = None,
            joined: List["Table"] = None) -> Dict[str, np.ndarray]:
        if joined is not None:
            return self.execute_joins(Plan(query), joined, group_hint)
        if right is not None:
            return self.execute_join(Plan(query), right, group_hint)
        return self.execute(Plan(query), group_hint)

    def free(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h:
            lib.nut_table_free(h)

    def __del__(self):
        self.free()
