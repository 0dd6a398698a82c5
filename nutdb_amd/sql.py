"""SQL front end and plan execution — Python mirror of the reference's interface.

The reference's only public API is ``nutdb::parser::Parser::parse(&str) ->
Result<Statement, ParseError>`` (src/lib.rs:3-4, src/parser/mod.rs:26-29).  Here the same
call goes through the C ABI (``nut_sql_parse``) into the C++ restatement of the
tokenizer/parser (nutdb_amd/csrc/sql_*.cpp):

    >>> Parser.parse("select a from t where a < 5").kind
    'Select'
    >>> Parser.parse("select a from t order by a asc")   # A8(i): ASC is never consumed
    Traceback (most recent call last):
    ParseError: Syntax Error: fail to parse (more than one statement) at line 1 col 28

``ParseError`` carries the reference's Display text ("Lex Error: ..." / "Syntax Error:
...", src/parser/error.rs:8-57) and ``lex`` (LexError vs SyntaxError).  Everything in
this module except ``execute`` runs on the CPU.
"""
from __future__ import annotations

import ctypes as C
import re
import json
from typing import Dict, List, Optional, Tuple

import numpy as np

from ._lib import (NUT_COL_HOST, NUT_OK, STMT_KINDS, TOKEN_TYPES, NutColumn, NutError, T_F64, T_I64, T_STR, check, lib)

NUT_ERR_PARSE = 6
NUT_ERR_CAPACITY = 5


class ParseError(Exception):
    """ParseError::{LexError, SyntaxError} (src/parser/error.rs:8-14)."""

    def __init__(self, message: str):
        super().__init__(message)
        self.message = message
        self.lex = message.startswith("Lex Error: ")


def _last_error() -> str:
    m = lib.nut_last_error()
    return m.decode() if m else ""


def _text(fn, handle) -> str:
    need = C.c_size_t(0)
    fn(handle, None, 0, C.byref(need))
    buf = C.create_string_buffer(need.value + 1)
    check(fn(handle, buf, len(buf), C.byref(need)), fn.__name__)
    return buf.value.decode()


class Statement:
    """A parsed statement (ast::Statement, src/parser/ast/mod.rs:13-24)."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)

    @property
    def kind(self) -> str:
        return STMT_KINDS[lib.nut_stmt_kind_of(self._h)]

    def dump(self) -> str:
        """S-expression of the tree (grammar: nutdb_amd/csrc/sql_dump.cpp)."""
        return _text(lib.nut_stmt_dump, self._h)

    def __repr__(self) -> str:
        return f"Statement({self.dump()})"

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            lib.nut_stmt_free(h)


class Parser:
    @staticmethod
    def parse(sql: str) -> Statement:
        """Parser::parse (src/parser/mod.rs:26-29): raises ParseError on rejection."""
        b = sql.encode("utf-8")
        h = C.c_void_p()
        st = lib.nut_sql_parse(b, len(b), C.byref(h))
        if st == NUT_ERR_PARSE:
            raise ParseError(_last_error())
        check(st, "nut_sql_parse")
        return Statement(h.value)


def tokenize(sql: str) -> List[Tuple[str, str]]:
    """Tokenizer::next_token until EOF (src/parser/tokenizer/mod.rs:66-112), whitespace and
    comment tokens included: [(TokenType name, token text)].  Raises ParseError on a
    lexical error."""
    b = sql.encode("utf-8")
    cap = len(b) + 2
    types = (C.c_int32 * cap)()
    spans = (C.c_uint64 * (2 * cap))()
    n = C.c_size_t(0)
    st = lib.nut_sql_tokenize(b, len(b), types, spans, cap, C.byref(n))
    if st == NUT_ERR_PARSE:
        raise ParseError("Lex Error: " + _last_error())
    check(st, "nut_sql_tokenize")
    return [(TOKEN_TYPES[types[i]], b[spans[2 * i]:spans[2 * i + 1]].decode()) for i in range(n.value)]


def _unescape(s: str, quote: str) -> str:
    b = s.encode("utf-8")
    cap = len(b) * 4 + 4
    out = C.create_string_buffer(cap)
    n = C.c_size_t(0)
    st = lib.nut_sql_unescape(b, len(b), ord(quote), out, cap, C.byref(n))
    if st == NUT_ERR_PARSE:
        raise ParseError(_last_error())
    check(st, "nut_sql_unescape")
    return out.raw[: n.value].decode()


def unescape_single_quoted_string(s: str) -> str:
    """src/parser/literal.rs:102"""
    return _unescape(s, "'")


def unescape_double_quoted_string(s: str) -> str:
    """src/parser/literal.rs:103"""
    return _unescape(s, '"')


def read_result(res) -> Dict[str, np.ndarray]:
    """nut_result -> {output name: numpy array} (NUT_T_STR columns: object arrays of str);
    a column holding SQL NULLs (nut_result_validity: a LEFT-joined table's column, a CASE
    without ELSE) is a numpy masked array, masked where NULL.  Frees the result."""
    try:
        nr = C.c_uint64(0)
        nc = C.c_int(0)
        check(lib.nut_result_shape(res, C.byref(nr), C.byref(nc)), "nut_result_shape")
        out = {}
        for j in range(nc.value):
            typ = C.c_int(0)
            nm = C.c_char_p()
            check(lib.nut_result_column(res, j, C.byref(typ), C.byref(nm)), "nut_result_column")
            if typ.value == T_STR:
                a = np.empty(nr.value, dtype=object)
                sp, sl = C.c_char_p(), C.c_size_t()
                for i in range(nr.value):
                    check(lib.nut_result_string(res, j, i, C.byref(sp), C.byref(sl)), "nut_result_string")
                    a[i] = C.string_at(sp, sl.value).decode("utf-8")
            else:
                a = np.empty(nr.value, dtype=np.float64 if typ.value == T_F64 else np.int64)
                check(lib.nut_result_to_host(res, j, a.ctypes.data_as(C.c_void_p), nr.value), "nut_result_to_host")
            vd = C.c_void_p()  # (any type: string columns hold NULLs too)
            check(lib.nut_result_validity(res, j, C.byref(vd)), "nut_result_validity")
            if vd.value:
                ok = np.empty(nr.value, dtype=np.uint8)
                check(lib.nut_result_validity_to_host(res, j, ok.ctypes.data_as(C.c_void_p), nr.value),
                      "nut_result_validity_to_host")
                a = np.ma.masked_array(a, mask=ok == 0)
            out[nm.value.decode()] = a
        return out
    finally:
        lib.nut_result_free(res)


class Plan:
    """An executor plan lowered from a SELECT."""

    KINDS = ["filter", "groupby", "sort"]

    def __init__(self, sql: str):
        b = sql.encode("utf-8")
        h = C.c_void_p()
        st = lib.nut_sql_plan(b, len(b), C.byref(h))
        if st == NUT_ERR_PARSE:
            raise ParseError(_last_error())
        check(st, "nut_sql_plan")
        self._h = h

    @property
    def kind(self) -> str:
        return self.KINDS[lib.nut_plan_kind_of(self._h)]

    def describe(self) -> dict:
        return json.loads(_text(lib.nut_plan_describe, self._h))

    @property
    def columns(self) -> List[str]:
        return self.describe()["columns"]

    def prepare(self, types: Dict[str, str]) -> None:
        """Compile an expression-mode plan's kernel ahead of execute (hipRTC, no GPU
        needed); `types` = {column: "int64" | "float64"}.  No-op for fused plans."""
        arr = (NutColumn * max(len(types), 1))()
        names = [k.encode() for k in types]
        for i, (name, t) in enumerate(types.items()):
            arr[i].name = names[i]
            arr[i].data = None
            arr[i].type = {"int64": T_I64, "float64": T_F64}[t]
        check(lib.nut_plan_prepare(self._h, arr, len(types)), "nut_plan_prepare")

    def route(self, types: Dict[str, str]) -> str:
        """The executor route over columns of these types (nut_plan_route: host only, no
        GPU) — e.g. "fused-sort", "rerun-expression -> expr-sort-f64-order"; raises the
        NutError execution would raise for a shape the executor rejects."""
        arr = (NutColumn * max(len(types), 1))()
        names = [k.encode() for k in types]
        for i, (name, t) in enumerate(types.items()):
            arr[i].name = names[i]
            arr[i].data = None
            arr[i].type = {"int64": T_I64, "float64": T_F64}[t]
        fn = lambda h, buf, cap, ln: lib.nut_plan_route(h, arr, len(types), buf, cap, ln)  # noqa: E731
        fn.__name__ = "nut_plan_route"
        return _text(fn, self._h)

    def execute(self, ex, columns: Dict[str, "object"], nrows: Optional[int] = None,
                group_hint: int = 0) -> Dict[str, np.ndarray]:
        """Run on the GPU of executor `ex` with `columns` = {name: 1-D int64/float64 CUDA
        tensor}.  Returns {output name: numpy array} in SELECT-list order."""
        arr, keep, n = self._bind(columns)
        rows = nrows if nrows is not None else (n or 0)
        res = C.c_void_p()
        ex._bind_stream()
        check(lib.nut_plan_execute(ex.ctx, self._h, arr, len(columns), rows, group_hint, C.byref(res)),
              "nut_plan_execute")
        return read_result(res)

    def execute_join(self, ex, left: Dict[str, "object"], right: Dict[str, "object"],
                     group_hint: int = 0) -> Dict[str, np.ndarray]:
        """Run a plan with a JOIN (nut_plan_execute2): `left` = the FROM table's columns,
        `right` = the JOIN source's (names unique across both).  The ON columns are
        int64; the hash join runs on the GPU and the rest of the plan on the joined rows."""
        la, lk, ln = self._bind(left)
        ra, rk, rn = self._bind(right)
        res = C.c_void_p()
        ex._bind_stream()
        check(lib.nut_plan_execute2(ex.ctx, self._h, la, len(left), ln or 0, ra, len(right), rn or 0,
                                    group_hint, C.byref(res)), "nut_plan_execute2")
        return read_result(res)

    def execute_tables(self, ex, tables: list, group_hint: int = 0) -> Dict[str, np.ndarray]:
        """A plan over several tables (nut_plan_executen): `tables` = [FROM columns, first
        JOIN source's columns, ...], each {name: CUDA tensor}."""
        bound = [self._bind(t) for t in tables]
        k = len(tables)
        arrs = (C.c_void_p * k)(*[C.cast(b[0], C.c_void_p) for b in bound])
        nco = (C.c_int * k)(*[len(t) for t in tables])
        nro = (C.c_uint64 * k)(*[b[2] or 0 for b in bound])
        res = C.c_void_p()
        ex._bind_stream()
        check(lib.nut_plan_executen(ex.ctx, self._h, arrs, nco, nro, k, group_hint, C.byref(res)), "nut_plan_executen")
        return read_result(res)

    def _bind(self, columns):
        import torch
        d = self.describe()
        # a subquery's columns are shown "subN:name" 
        names = [re.sub(r"^sub\d+:", "", c) for c in d["columns"]]
        star = d.get("column") == "*"  # SELECT *: every column given is projected
        arr = (NutColumn * max(len(columns), 1))()
        keep = []
        n = None
        for i, (name, t) in enumerate(columns.items()):
            host = isinstance(t, np.ndarray) or (isinstance(t, torch.Tensor) and not t.is_cuda)
            if host:  # host memory: the library copies it into HBM for the call (NUT_COL_HOST)
                t = torch.from_numpy(np.ascontiguousarray(t)) if isinstance(t, np.ndarray) else t.contiguous()
                keep.append(t)
            if not isinstance(t, torch.Tensor) or t.dim() != 1 or not t.is_contiguous():
                raise ValueError(f"column {name!r} must be a contiguous 1-D CUDA tensor or host array")
            if t.dtype == torch.int64:
                typ = T_I64
            elif t.dtype == torch.float64:
                typ = T_F64
            else:
                raise ValueError(f"column {name!r}: dtype {t.dtype} is not int64/float64")
            nb = name.encode()
            keep.append(nb)
            arr[i] = NutColumn(nb, t.data_ptr(), typ | (NUT_COL_HOST if host else 0))
            low = name.lower()
            if star or any(low == c.lower() or c.lower().endswith("." + low) for c in names):  # JOIN plans qualify
                n = t.numel() if n is None else n
                if t.numel() != n:
                    raise ValueError("bound columns differ in length")
        return arr, keep, n

    def _handle(self):
        return self._h

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            lib.nut_plan_free(h)


__all__ = ["ParseError", "Parser", "Plan", "Statement", "tokenize", "unescape_single_quoted_string",
           "unescape_double_quoted_string", "NutError", "NUT_OK"]
