"""Expression-program oracle (numpy) — TEST INFRASTRUCTURE ONLY.

Restates the semantics of include/nutexec.h `nut_prog` (RPN expression programs, the
expression mode of nut_groupby; nutdb_amd/csrc/jit.cpp generates the device code)
column-at-a-time with numpy, independently of the generated HIP code:

  * i64 + - * wrap (two's complement); any f64 operand makes the op f64 (the int is
    converted with round-to-nearest); DIV is always f64;
  * MOD / INTDIV on ints truncate toward zero; a zero divisor is an error of the row;
    INT64_MIN % -1 = 0 and INT64_MIN div -1 wraps; MOD on f64 is C fmod;
  * comparisons give bool; int vs f64 compares as f64; NaN compares unequal;
  * AND / OR / XOR / NOT over bools (ints: non-zero = true), both operands evaluated;
  * bit ops and shifts on ints; shift counts outside [0, 63] give 0 (SHR of a
    negative value: -1); SHR is arithmetic;
  * IF takes the chosen branch's value and only the chosen branch's errors;
  * DATEPART (arg = nut_date_part) of a day number (days since 1970-01-01, clamped to
    +-2^40): proleptic Gregorian civil-from-days with truncating division.

Errors are tracked per row (a bool array); the group-by rule is the kernel's
(agg_kernel.hpp consume_rows): a WHERE error counts for every row, an aggregate's mask
error for rows passing WHERE, its value error for rows passing WHERE and its mask.

The reference (nutdb v0.1.0) executes no expressions at all — it stops at the AST
 — so these semantics are defined by this build and the oracle is
"parity unpinned" with respect to the reference; the SQL→program lowering they are fed
from is pinned by the front-end tests against the reference's own fixtures.
"""
from __future__ import annotations

import numpy as np

OPS = ["col", "i64", "f64", "add", "sub", "mul", "div", "mod", "intdiv", "lt", "le", "gt", "ge", "eq", "ne",
       "and", "or", "xor", "not", "bitand", "bitor", "bitxor", "bitnot", "shl", "shr", "if", "abs", "to_f64",
       "lookup", "datepart"]
OP = {name: i for i, name in enumerate(OPS)}
I64, F64, BOOL = 0, 1, 2
_ARITY = {OP["not"]: 1, OP["bitnot"]: 1, OP["abs"]: 1, OP["to_f64"]: 1, OP["if"]: 3, OP["lookup"]: 1,
          OP["datepart"]: 1}
DP_YEAR, DP_MONTH, DP_DAY, DP_QUARTER, DP_WEEKDAY, DP_YEARDAY, DP_YYYYMM, DP_YYYYMMDD = range(8)


def _tdiv(a, b: int):
    """int64 division truncating toward zero by a positive constant b."""
    q = np.floor_divide(a, b)
    return q + ((a - q * b != 0) & (a < 0))


def date_part(days, part: int):
    """nut_date_part `part` of day numbers (int64 array), as nut_prog DATEPART computes it."""
    d = np.clip(np.asarray(days, dtype=np.int64), -(1 << 40), 1 << 40)
    z = d + 719468
    era = _tdiv(np.where(z >= 0, z, z - 146096), 146097)
    doe = z - era * 146097
    yoe = _tdiv(doe - _tdiv(doe, 1460) + _tdiv(doe, 36524) - _tdiv(doe, 146096), 365)
    doy = doe - (365 * yoe + _tdiv(yoe, 4) - _tdiv(yoe, 100))
    mp = _tdiv(5 * doy + 2, 153)
    m = np.where(mp < 10, mp + 3, mp - 9)
    y = yoe + era * 400 + (m <= 2)
    if part == DP_YEAR:
        return y
    if part == DP_MONTH:
        return m
    if part == DP_DAY:
        return doy - _tdiv(153 * mp + 2, 5) + 1
    if part == DP_QUARTER:
        return _tdiv(m - 1, 3) + 1
    if part == DP_WEEKDAY:
        return (d + 3) % 7 + 1  # numpy % is floor-mod: 1970-01-01 (day 0) is a Thursday (4)
    if part == DP_YEARDAY:
        leap = ((y % 4 == 0) & (y % 100 != 0)) | (y % 400 == 0)
        return np.where(doy >= 306, doy - 305, doy + 60 + leap)
    if part == DP_YYYYMM:
        return y * 100 + m
    if part == DP_YYYYMMDD:
        return y * 10000 + m * 100 + (doy - _tdiv(153 * mp + 2, 5) + 1)
    raise ProgramError(f"unknown date part {part}")


class ProgramError(ValueError):
    pass


class DivisionByZero(ArithmeticError):
    pass


def _f(v):
    x, t, _ = v
    return x if t == F64 else x.astype(np.float64)


def _i(v):
    x, t, _ = v
    if t == F64:
        raise ProgramError("integer operand expected, got float64")
    return x.astype(np.int64)


def _b(v):
    x, t, _ = v
    if t == F64:
        raise ProgramError("boolean or integer operand expected, got float64")
    return x.astype(bool) if t == BOOL else x != 0


def eval_prog(nodes, cols, n=None):
    """nodes: [(op, arg, v)] (op index or name; v = int64 constant or the double's bits);
    cols: list of int64 / float64 arrays.  Returns (values, type, err): values int64
    (I64/BOOL as 0/1) or float64, type I64/F64/BOOL, err a bool array."""
    if n is None:
        n = len(cols[0]) if cols else 0
    st = []
    z = np.zeros(n, dtype=bool)
    with np.errstate(all="ignore"):
        for node in nodes:
            op, arg, v = (tuple(node) + (0, 0))[:3]
            op = OP[op] if isinstance(op, str) else int(op)
            if op == OP["f64"] and isinstance(v, float):
                v = int(np.array([v], dtype=np.float64).view(np.int64)[0])
            k = 0 if op <= OP["f64"] else _ARITY.get(op, 2)
            if len(st) < k:
                raise ProgramError("stack underflow")
            a = st[len(st) - k:]
            del st[len(st) - k:]
            err = z.copy()
            for x in a:
                err = err | x[2]
            f = k == 2 and (a[0][1] == F64 or a[1][1] == F64)
            if op == OP["col"]:
                c = np.asarray(cols[arg])
                r = (c.astype(np.float64), F64) if c.dtype == np.float64 else (c.astype(np.int64), I64)
            elif op == OP["i64"]:
                r = (np.full(n, v, dtype=np.int64), I64)
            elif op == OP["f64"]:
                r = (np.full(n, np.int64(v).view(np.float64), dtype=np.float64), F64)
            elif op in (OP["add"], OP["sub"], OP["mul"]):
                fn = {OP["add"]: np.add, OP["sub"]: np.subtract, OP["mul"]: np.multiply}[op]
                r = (fn(_f(a[0]), _f(a[1])), F64) if f else (fn(_i(a[0]), _i(a[1])), I64)
            elif op == OP["div"]:
                r = (np.divide(_f(a[0]), _f(a[1])), F64)
            elif op in (OP["mod"], OP["intdiv"]):
                if f:
                    if op == OP["intdiv"]:
                        raise ProgramError("integer division needs integer operands")
                    r = (np.fmod(_f(a[0]), _f(a[1])), F64)
                else:
                    x, y = _i(a[0]), _i(a[1])
                    zero, m1 = y == 0, y == -1
                    ys = np.where(zero | m1, 1, y)
                    q = np.floor_divide(x, ys)
                    rem = x - q * ys
                    fix = (rem != 0) & ((x < 0) != (ys < 0))  # floor -> truncation
                    q = np.where(fix, q + 1, q)
                    rem = np.where(fix, rem - ys, rem)
                    if op == OP["mod"]:
                        out = np.where(zero | m1, 0, rem)
                    else:
                        out = np.where(zero, 0, np.where(m1, np.negative(x), q))
                    r = (out.astype(np.int64), I64)
                    err = err | zero
            elif OP["lt"] <= op <= OP["ne"]:
                fn = [np.less, np.less_equal, np.greater, np.greater_equal, np.equal, np.not_equal][op - OP["lt"]]
                r = (fn(_f(a[0]), _f(a[1])) if f else fn(_i(a[0]), _i(a[1])), BOOL)
            elif op in (OP["and"], OP["or"], OP["xor"]):
                fn = {OP["and"]: np.logical_and, OP["or"]: np.logical_or, OP["xor"]: np.not_equal}[op]
                r = (fn(_b(a[0]), _b(a[1])), BOOL)
            elif op == OP["not"]:
                r = (~_b(a[0]), BOOL)
            elif op in (OP["bitand"], OP["bitor"], OP["bitxor"]):
                if f:
                    raise ProgramError("bitwise operators need integer operands")
                fn = {OP["bitand"]: np.bitwise_and, OP["bitor"]: np.bitwise_or, OP["bitxor"]: np.bitwise_xor}[op]
                r = (fn(_i(a[0]), _i(a[1])), I64)
            elif op == OP["bitnot"]:
                r = (np.invert(_i(a[0])), I64)
            elif op in (OP["shl"], OP["shr"]):
                if f:
                    raise ProgramError("bitwise operators need integer operands")
                x, y = _i(a[0]), _i(a[1])
                ok = (y >= 0) & (y < 64)
                ys = np.where(ok, y, 0).astype(np.uint64)
                if op == OP["shl"]:
                    out = np.where(ok, np.left_shift(x.view(np.uint64), ys).view(np.int64), 0)
                else:
                    out = np.where(ok, np.right_shift(x, ys.astype(np.int64)), np.where(x < 0, -1, 0))
                r = (out.astype(np.int64), I64)
            elif op == OP["if"]:
                c = _b(a[0])
                x, y = a[1], a[2]
                if x[1] == BOOL and y[1] == BOOL:
                    r = (np.where(c, _b(x), _b(y)), BOOL)
                elif x[1] == F64 or y[1] == F64:
                    r = (np.where(c, _f(x), _f(y)), F64)
                else:
                    r = (np.where(c, _i(x), _i(y)), I64)
                err = a[0][2] | np.where(c, x[2], y[2])
            elif op == OP["abs"]:
                r = (np.abs(_f(a[0])), F64) if a[0][1] == F64 else (np.abs(_i(a[0])), I64)
            elif op == OP["to_f64"]:
                r = (_f(a[0]), F64)
            elif op == OP["datepart"]:
                r = (date_part(_i(a[0]), int(arg)).astype(np.int64), I64)
            else:
                raise ProgramError(f"unknown op {op}")
            st.append((r[0], r[1], err))
    if len(st) != 1:
        raise ProgramError(f"program leaves {len(st)} values")
    x, t, err = st[0]
    if t == BOOL:
        x = x.astype(np.int64)
    return x, t, err


def eval_prog_par(nodes, cols, n=None, threads=1):
    """eval_prog over row chunks on `threads` host threads (numpy releases the GIL in its
    array loops).  Programs are row-wise, so the result is eval_prog's, bit for bit; the
    CPU baseline (bench.py) uses it to run the expression oracle on every host core."""
    if n is None:
        n = len(cols[0]) if cols else 0
    if threads <= 1 or n < (1 << 20):
        return eval_prog(nodes, cols, n)
    from concurrent.futures import ThreadPoolExecutor
    bounds = [n * i // threads for i in range(threads + 1)]
    with ThreadPoolExecutor(threads) as pool:
        parts = list(pool.map(lambda lh: eval_prog(nodes, [c[lh[0]:lh[1]] for c in cols], lh[1] - lh[0]),
                              zip(bounds[:-1], bounds[1:])))
    return np.concatenate([p[0] for p in parts]), parts[0][1], np.concatenate([p[2] for p in parts])


def groupby_prog(keys, cols, where, aggs, n=None, threads=1, engine="numpy"):
    """Expression-mode group-by: keys = list of int64 arrays or key programs (node lists,
    int64 / bool; any number of keys; empty = global aggregate), where = nodes or None,
    aggs = [(op, val_nodes or None, mask_nodes or None)] with op 0 SUM / 1 COUNT / 2 MIN /
    3 MAX.  Returns (keys, words, types) like oracle.groupby (words = result bits, groups
    ordered by key tuple) plus each aggregate's value type; raises DivisionByZero under the
    kernel's error rule (a key program's error counts for rows passing WHERE).  threads > 1:
    the programs run on that many host threads (eval_prog_par; same result).  engine "c":
    integer / bool programs run in C on every core (oracle.eval_int, no row errors possible
    in that subset; pinned to eval_prog by tests/test_expr_cpu.py), the rest as above —
    the CPU baseline's form."""
    from . import oracle as orc

    def eval_prog(nodes, cols, n):  # noqa: F811  (the row-chunked / C forms)
        if engine == "c" and n and cols:
            x = orc.eval_int(nodes, cols, n)
            if x is not None:  # the type from one row of the numpy form
                return x, _eval_numpy(nodes, [c[:1] for c in cols], 1)[1], np.zeros(n, dtype=bool)
        return eval_prog_par(nodes, cols, n, threads)

    if n is None:
        arrs = [k for k in keys if isinstance(k, np.ndarray)]
        n = len(arrs[0]) if arrs else len(cols[0])
    ok = np.ones(n, dtype=bool)
    bad = np.zeros(n, dtype=bool)
    if where:
        w, t, e = eval_prog(where, cols, n)
        if t == F64:
            raise ProgramError("WHERE is float64")
        ok = w != 0
        bad |= e
    kv = []
    for k in keys:
        if isinstance(k, np.ndarray):
            kv.append(k.astype(np.int64))
            continue
        x, t, e = eval_prog(k, cols, n)
        if t == F64:
            raise ProgramError("float64 key program")
        bad |= ok & e
        kv.append(x.astype(np.int64))
    keys = kv
    values, masks, spec, types = [], [], [], []
    for a, (op, val, mask) in enumerate(aggs):
        m = None
        if mask:
            mv, mt, me = eval_prog(mask, cols, n)
            m = mv != 0
            bad |= ok & me
        take = ok if m is None else ok & m
        if op == 1:
            types.append(I64)
            spec.append((1, 0, ()))
        else:
            v, t, e = eval_prog(val, cols, n)
            bad |= take & e
            types.append(t)
            values.append(v)
            spec.append((op, 0, (len(values) - 1,)))
        masks.append(m)
    if bad.any():
        raise DivisionByZero("division by zero in an expression")
    kk = list(keys) if keys else [np.zeros(n, dtype=np.int64)]
    if len(kk) <= 2:
        ok_keys, words = orc.groupby(kk, spec, values=values, row_mask=ok, agg_masks=masks)
        return ok_keys, words, types
    # more keys than the C oracle takes: the tuple's rank among the distinct tuples (numpy
    # sorts them lexicographically) is one key with the same grouping and order
    tup = np.stack(kk, axis=1)
    uniq, rank = np.unique(tup, axis=0, return_inverse=True)
    ok_rank, words = orc.groupby([rank.reshape(-1).astype(np.int64)], spec, values=values, row_mask=ok,
                                 agg_masks=masks)
    return uniq[ok_rank[:, 0]], words, types


_eval_numpy = eval_prog
