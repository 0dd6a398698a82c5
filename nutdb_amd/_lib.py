"""ctypes binding of libnutexec.so — the C ABI declared in include/nutexec.h.

This is the same binding a Rust host would write with `extern "C"`:
plain integers, doubles and pointers.  The library is REQUIRED: if it is missing or
fails to load, importing nutdb_amd raises — there is no CPU fallback anywhere in the
product path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

# torch must own the HIP runtime before libnutexec.so resolves libamdhip64.so.7, so
# that torch-allocated device pointers and the library share one runtime/context.
import torch  # noqa: F401

LIB_PATH = Path(os.environ.get("NUTEXEC_LIB", Path(__file__).resolve().parent / "libnutexec.so"))

NUT_MAX_KEYS = 2
NUT_MAX_PRED = 6
NUT_MAX_VALS = 4
NUT_MAX_AGGS = 8
NUT_MAX_SET = 16
NUT_MAX_PROG_COLS = 16
NUT_MAX_PROG_NODES = 256

# nut_status
NUT_OK = 0
NUT_ERR_CAPACITY = 5
NUT_JOIN_ANY_ORDER = 0x100
NUT_COL_HOST = 0x100
STATUS_NAMES = {
    0: "NUT_OK", 1: "NUT_ERR_INVALID_ARG", 2: "NUT_ERR_HIP", 3: "NUT_ERR_OOM",
    4: "NUT_ERR_UNSUPPORTED", 5: "NUT_ERR_CAPACITY", 6: "NUT_ERR_PARSE", 7: "NUT_ERR_PLAN",
    8: "NUT_ERR_TIMEOUT",
}

# enums (include/nutexec.h)
GEN_U62, GEN_FULL_I64, GEN_POOL_KEY, GEN_DYADIC, GEN_UNIT_F64, GEN_RANGE_I64, GEN_RANGE_F64, GEN_SKEW_KEY = range(8)
LT, LE, GT, GE, EQ, NE, IN, NOT_IN = range(8)
T_I64, T_F64, T_STR = 0, 1, 2
COL_KINDS = ["int", "uint", "float", "bool", "date", "datetime", "string", "enum"]
KERNEL_FILTER, KERNEL_AGGREGATE, KERNEL_SORT = 0, 1, 2
AGG_SUM, AGG_COUNT, AGG_MIN, AGG_MAX = range(4)
EX_COL, EX_MUL, EX_ADD, EX_SUB, EX_MUL_1M, EX_MUL_1M_1P = range(6)
# nut_prog_op (expression programs, RPN) and nut_prog_value_type
PROG_OPS = ["col", "i64", "f64", "add", "sub", "mul", "div", "mod", "intdiv", "lt", "le", "gt", "ge", "eq", "ne",
            "and", "or", "xor", "not", "bitand", "bitor", "bitxor", "bitnot", "shl", "shr", "if", "abs", "to_f64", "lookup",
            "datepart"]
# nut_date_part (the arg of a "datepart" node)
DP_YEAR, DP_MONTH, DP_DAY, DP_QUARTER, DP_WEEKDAY, DP_YEARDAY, DP_YYYYMM, DP_YYYYMMDD = range(8)
P = {name: i for i, name in enumerate(PROG_OPS)}
PT_I64, PT_F64, PT_BOOL = 0, 1, 2


class NutProgNode(C.Structure):
    _fields_ = [("op", C.c_int32), ("arg", C.c_int32), ("v", C.c_int64)]


class NutProg(C.Structure):
    _fields_ = [("n", C.c_int32), ("node", C.POINTER(NutProgNode))]


class NutAggSpec(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("nkeys", C.c_int32),
        ("keys", C.c_void_p * NUT_MAX_KEYS),
        ("npred", C.c_int32),
        ("pred_col", C.c_void_p * NUT_MAX_PRED),
        ("pred_type", C.c_int32 * NUT_MAX_PRED),
        ("pred_op", C.c_int32 * NUT_MAX_PRED),
        ("pred_i64", C.c_int64 * NUT_MAX_PRED),
        ("pred_f64", C.c_double * NUT_MAX_PRED),
        ("nvals", C.c_int32),
        ("val_col", C.c_void_p * NUT_MAX_VALS),
        ("val_type", C.c_int32 * NUT_MAX_VALS),
        ("naggs", C.c_int32),
        ("agg_op", C.c_int32 * NUT_MAX_AGGS),
        ("agg_expr", C.c_int32 * NUT_MAX_AGGS),
        ("agg_arg", (C.c_int32 * 3) * NUT_MAX_AGGS),
        ("pred_nset", C.c_int32 * NUT_MAX_PRED),
        ("pred_set", (C.c_int64 * NUT_MAX_SET) * NUT_MAX_PRED),
        ("prog_mode", C.c_int32),
        ("nprog_cols", C.c_int32),
        ("prog_col", C.c_void_p * NUT_MAX_PROG_COLS),
        ("prog_col_type", C.c_int32 * NUT_MAX_PROG_COLS),
        ("where", NutProg),
        ("agg_val", NutProg * NUT_MAX_AGGS),
        ("agg_mask", NutProg * NUT_MAX_AGGS),
        ("key_prog", NutProg * NUT_MAX_KEYS),
    ]


class NutColumn(C.Structure):
    """nut_column: a named device column bound to a plan at execute time."""
    _fields_ = [("name", C.c_char_p), ("data", C.c_void_p), ("type", C.c_int32)]


PLAN_FILTER, PLAN_GROUPBY, PLAN_SORT = 0, 1, 2
STMT_KINDS = ["Select", "Insert", "Explain", "Alter", "Create", "Describe", "Drop", "Truncate", "Optimize", "Set"]
# TokenType order (reference src/parser/tokenizer/token.rs:5-91)
TOKEN_TYPES = [
    "KeywordOrIdentifier", "DelimitedIdentifier", "ConfigIdentifier", "QueryParameter", "RawStringLiteral",
    "EscapedSQStringLiteral", "EscapedDQStringLiteral", "IntegerLiteral", "FloatLiteral", "HexLiteral", "Comma",
    "Dot", "Colon", "SemiColon", "Plus", "Minus", "Mul", "Div", "Mod", "Eq", "NotEq", "Lt", "Gt", "LtEq", "GtEq",
    "LParen", "RParen", "LBracket", "RBracket", "LBrace", "RBrace", "BitAnd", "BitOr", "BitXor", "BitNot",
    "BitLShift", "BitRShift", "Comment", "Whitespace", "EOF",
]


class NutError(RuntimeError):
    def __init__(self, status: int, where: str, message: str):
        self.status = status
        self.name = STATUS_NAMES.get(status, f"status {status}")
        super().__init__(f"{where}: {self.name}: {message}")


# name -> (restype, argtypes)
_P = C.c_void_p
_U64 = C.c_uint64
_I64 = C.c_int64
_I32 = C.c_int
SIGNATURES = {
    "nut_abi_version": (_I32, []),
    "nut_last_error": (C.c_char_p, []),
    "nut_ctx_create": (_I32, [_I32, C.POINTER(_P)]),
    "nut_ctx_destroy": (None, [_P]),
    "nut_ctx_set_stream": (_I32, [_P, _P]),
    "nut_ctx_sync": (_I32, [_P]),
    "nut_ctx_info": (_I32, [_P, C.POINTER(_I32), C.c_char_p, C.c_size_t]),
    "nut_ctx_enable_timing": (_I32, [_P, _I32]),
    "nut_ctx_kernel_time": (_I32, [_P, _I32, C.POINTER(C.c_double), C.POINTER(_U64)]),
    "nut_ctx_sort_stats": (_I32, [_P, C.POINTER(_U64), C.POINTER(C.c_uint32)]),
    "nut_ctx_groupby_stats": (_I32, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "nut_ctx_groupby_overflow": (_I32, [_P, C.POINTER(_U64), C.POINTER(C.c_uint32)]),
    "nut_ctx_groupby_heavy": (_I32, [_P, C.POINTER(C.c_uint32), C.POINTER(_U64)]),
    "nut_ctx_priv_shape": (_I32, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double)]),
    "nut_ctx_priv_probe_cost": (_I32, [_P, C.POINTER(C.c_double)]),
    "nut_ctx_set_option": (_I32, [_P, _I32, _I64]),
    "nut_ctx_get_option": (_I32, [_P, _I32, C.POINTER(_I64)]),
    "nut_join_i64": (_I32, [_P, _P, _U64, _P, _U64, _I32, C.POINTER(_P), C.POINTER(_U64)]),
    "nut_join_write": (_I32, [_P, _P, _P]),
    "nut_join_i64_into": (_I32, [_P, _P, _U64, _P, _U64, _I32, _P, _P, _U64, C.POINTER(_U64)]),
    "nut_join_free": (None, [_P]),
    "nut_hash_partition_i64": (_I32, [_P, _P, _U64, _I32, _I64, _P, _P, C.POINTER(_U64)]),
    "nut_gather_u64": (_I32, [_P, _P, _P, _U64, _U64, _P]),
    "nut_select_rows": (_I32, [_P, C.POINTER(NutAggSpec), _P, C.POINTER(_U64)]),
    "nut_select_jit_compile": (_I32, [C.POINTER(NutAggSpec)]),
    "nut_eval_rows": (_I32, [_P, C.POINTER(NutAggSpec), _P, _U64, _P, _P]),
    "nut_eval_jit_compile": (_I32, [C.POINTER(NutAggSpec)]),
    "nut_gen_column": (_I32, [_P, _I32, _U64, _I64, _I64, C.c_double, _U64, _U64, _P]),
    "nut_stream_probe": (_I32, [_P, _P, _U64, _P, _U64, _I32, C.POINTER(C.c_double)]),
    "nut_filter_i64": (_I32, [_P, _P, _U64, _I32, _I64, _P, C.POINTER(_U64)]),
    "nut_filter_i64_async": (_I32, [_P, _P, _U64, _I32, _I64, _P, _P]),
    "nut_groupby": (_I32, [_P, C.POINTER(NutAggSpec), _U64, C.POINTER(_P)]),
    "nut_groupby_accumulate": (_I32, [_P, C.POINTER(NutAggSpec), _P]),
    "nut_prog_type": (_I32, [C.POINTER(NutProg), C.POINTER(C.c_int32), _I32, C.POINTER(C.c_int32)]),
    "nut_groupby_jit_source": (_I32, [C.POINTER(NutAggSpec), C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "nut_groupby_jit_compile": (_I32, [C.POINTER(NutAggSpec)]),
    "nut_plan_prepare": (_I32, [_P, C.POINTER(NutColumn), _I32]),
    "nut_result_string": (_I32, [_P, _I32, _U64, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t)]),
    "nut_table_create": (_I32, [C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    "nut_table_shape": (_I32, [_P, C.POINTER(_I32), C.POINTER(_U64)]),
    "nut_table_column_info": (_I32, [_P, _I32, C.POINTER(C.c_char_p), C.POINTER(_I32), C.POINTER(_I32),
                                     C.POINTER(_I32)]),
    "nut_table_append": (_I32, [_P, _P, _I32, _P, _P, _U64]),
    "nut_table_execute": (_I32, [_P, _P, _P, _U64, C.POINTER(_P)]),
    "nut_table_execute2": (_I32, [_P, _P, _P, _P, _U64, C.POINTER(_P)]),
    "nut_table_executen": (_I32, [_P, C.POINTER(_P), _I32, _P, _U64, C.POINTER(_P)]),
    "nut_table_free": (None, [_P]),
    "nut_groups_size": (_I32, [_P, C.POINTER(_U64)]),
    "nut_groups_to_host": (_I32, [_P, _P, _P, _U64]),
    "nut_groups_to_device": (_I32, [_P, _P, _U64]),
    "nut_groups_partition": (_I32, [_P, _I32, _P, _U64, C.POINTER(_U64)]),
    "nut_groups_free": (None, [_P]),
    "nut_groupby_to_host": (_I32, [_P, C.POINTER(NutAggSpec), _U64, _P, _P, _U64, C.POINTER(_U64)]),
    "nut_groupby_i64_f64": (_I32, [_P, _P, _P, _U64, C.c_uint32, _U64, C.POINTER(_P)]),
    "nut_q1": (_I32, [_P, _P, _P, _P, _P, _P, _P, _U64, _I64, C.POINTER(_P)]),
    "nut_sort_i64": (_I32, [_P, _P, _P, _U64]),
    "nut_sort_i64_desc": (_I32, [_P, _P, _P, _U64]),
    "nut_partition_i64": (_I32, [_P, _P, _U64, _P, _I32, _P, _P]),
    # SQL front end (CPU) and plan lowering / execution
    "nut_sql_parse": (_I32, [C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    "nut_stmt_kind_of": (_I32, [_P]),
    "nut_stmt_dump": (_I32, [_P, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "nut_stmt_free": (None, [_P]),
    "nut_sql_tokenize": (_I32, [C.c_char_p, C.c_size_t, C.POINTER(C.c_int32), C.POINTER(_U64), C.c_size_t,
                                C.POINTER(C.c_size_t)]),
    "nut_sql_unescape": (_I32, [C.c_char_p, C.c_size_t, _I32, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "nut_sql_plan": (_I32, [C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    "nut_plan_kind_of": (_I32, [_P]),
    "nut_plan_describe": (_I32, [_P, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "nut_plan_route": (_I32, [_P, _P, _I32, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "nut_plan_free": (None, [_P]),
    "nut_plan_execute": (_I32, [_P, _P, _P, _I32, _U64, _U64, C.POINTER(_P)]),
    "nut_plan_execute2": (_I32, [_P, _P, _P, _I32, _U64, _P, _I32, _U64, _U64, C.POINTER(_P)]),
    "nut_plan_executen": (_I32, [_P, _P, C.POINTER(_P), C.POINTER(_I32), C.POINTER(_U64), _I32, _U64, C.POINTER(_P)]),
    "nut_result_shape": (_I32, [_P, C.POINTER(_U64), C.POINTER(_I32)]),
    "nut_result_column": (_I32, [_P, _I32, C.POINTER(_I32), C.POINTER(C.c_char_p)]),
    "nut_result_to_host": (_I32, [_P, _I32, _P, _U64]),
    "nut_result_device": (_I32, [_P, C.POINTER(_P)]),
    "nut_result_device_column": (_I32, [_P, _I32, C.POINTER(_P)]),
    "nut_result_validity": (_I32, [_P, _I32, C.POINTER(_P)]),
    "nut_result_validity_to_host": (_I32, [_P, _I32, _P, _U64]),
    "nut_result_free": (None, [_P]),
    "nut_ctx_memcpy": (_I32, [_P, _P, _P, C.c_size_t]),
    "nut_sort_pairs": (_I32, [_P, _P, _I32, _I32, _P, _P, _U64]),
    "nut_topk_positions": (_I32, [_P, _P, _I32, _I32, _U64, _U64, _P, _U64, C.POINTER(C.c_uint64)]),
    # multi-GPU (RCCL inside the library)
    "nut_dist_create": (_I32, [_I32, C.POINTER(_I32), C.POINTER(_P)]),
    "nut_dist_unique_id": (_I32, [_P]),
    "nut_dist_create_rank": (_I32, [_I32, _I32, _P, _I32, C.POINTER(_P)]),
    "nut_dist_create_virtual": (_I32, [_I32, _I32, C.POINTER(_P)]),
    "nut_dist_info": (_I32, [_P, C.POINTER(_I32), C.POINTER(_I32), C.POINTER(_I32)]),
    "nut_dist_ctx": (_P, [_P, _I32]),
    "nut_dist_destroy": (None, [_P]),
    "nut_dist_groupby": (_I32, [_P, _P, _U64, C.POINTER(_P)]),
    "nut_dist_sort_i64": (_I32, [_P, C.POINTER(_P), C.POINTER(_U64), C.POINTER(_P), C.POINTER(_U64)]),
    "nut_dist_filter_i64": (_I32, [_P, C.POINTER(_P), C.POINTER(_U64), _I32, _I64, C.POINTER(_P), C.POINTER(_U64),
                                   C.POINTER(_U64)]),
    "nut_dist_join_i64": (_I32, [_P, C.POINTER(_P), C.POINTER(_U64), C.POINTER(_I64), C.POINTER(_P), C.POINTER(_U64),
                                 C.POINTER(_I64), _I32, C.POINTER(_P), C.POINTER(_P), C.POINTER(_U64)]),
}
NUT_DIST_ID_BYTES = 128


def _load() -> C.CDLL:
    if not LIB_PATH.exists():
        raise ImportError(
            f"nutdb_amd: {LIB_PATH} is missing — build it with `python -m nutdb_amd.build` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback."
        )
    lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError here = ABI mismatch, fail loudly
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(status: int, where: str) -> None:
    if status != NUT_OK:
        msg = lib.nut_last_error()
        raise NutError(status, where, msg.decode() if msg else "")
