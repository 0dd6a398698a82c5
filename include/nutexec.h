/*
 * nutexec.h — C ABI of the MI355X-native columnar executor for NutDB.
 *
 * Drop-in boundary.  The reference crate (nutdb v0.1.0) stops at
 * `Parser::parse(sql) -> Result<Statement, ParseError>` (src/parser/mod.rs:26-29) and
 * has NO executor, plugin registry or FFI to slot behind; its AST nodes
 *   QueryBody.r#where   src/parser/ast/query.rs:30   (WhereClause, :68-72)
 *   QueryBody.group_by  src/parser/ast/query.rs:31   (GroupByClause, :74-78)
 *   QueryBody.columns   src/parser/ast/query.rs:25   (FnCall sum/count/min/max, expr.rs:32-36)
 *   QueryBody.order_by  src/parser/ast/query.rs:33   (OrderByClause, :86-90)
 * are what an executor lowers from.  Every entry point below is therefore the
 * replacement for an interface the reference does not yet have; each names the
 * AST node(s) it executes.  The Rust binding a maintainer would add is in
 * INTEGRATION.md.
 *
 * Conventions
 *  - Plain C: no C++ or torch types cross this boundary.
 *  - Column pointers are DEVICE pointers (HBM-resident columns; hipMalloc'd or
 *    torch-allocated) unless a parameter says "_host".
 *  - The caller owns column and output buffers; the library owns its scratch and
 *    the nut_groups result objects (freed by nut_groups_free).
 *  - Calls are ordered on the context's stream (nut_ctx_set_stream; default: a
 *    stream the context creates).  Entry points that return a host-visible value
 *    synchronise that stream before returning; "_async" variants do not.
 *  - Status is an int enum (0 = NUT_OK); nut_last_error() is a thread-local
 *    message describing the last failure on this thread (like the reference's
 *    thiserror messages, src/parser/error.rs:8-57).
 *  - One context per host thread per device.
 */
#ifndef NUTEXEC_H
#define NUTEXEC_H

#ifndef __HIPCC_RTC__ /* the runtime-compiled scan kernels bring their own */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define NUTEXEC_ABI_VERSION 1

typedef enum {
  NUT_OK = 0,
  NUT_ERR_INVALID_ARG = 1,
  NUT_ERR_HIP = 2,          /* HIP runtime / launch failure */
  NUT_ERR_OOM = 3,
  NUT_ERR_UNSUPPORTED = 4,  /* valid request outside what the kernels implement */
  NUT_ERR_CAPACITY = 5,     /* caller-provided output too small */
  NUT_ERR_PARSE = 6,        /* SQL rejected by the front end (LexError/SyntaxError) */
  NUT_ERR_PLAN = 7,         /* SQL parsed but cannot be lowered to an executor plan */
  NUT_ERR_TIMEOUT = 8       /* a bounded device-side spin expired (never expected) */
} nut_status;

typedef struct nut_ctx nut_ctx;
typedef struct nut_groups nut_groups;

int nut_abi_version(void);
const char *nut_last_error(void);

nut_status nut_ctx_create(int device, nut_ctx **out);
void nut_ctx_destroy(nut_ctx *ctx);
/* hip_stream is a hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL
 * selects the device's default (null) stream.  A new context starts on a stream of
 * its own. */
nut_status nut_ctx_set_stream(nut_ctx *ctx, void *hip_stream);
nut_status nut_ctx_sync(nut_ctx *ctx);
/* copy `bytes` between any host / device addresses on the context's stream and wait for
 * it (lets a host without its own HIP binding read library-owned device results) */
nut_status nut_ctx_memcpy(nut_ctx *ctx, void *dst, const void *src, size_t bytes);
/* number of CUs and device name, for reports */
nut_status nut_ctx_info(nut_ctx *ctx, int *num_cus, char *name, size_t name_len);

/* Device-side timing of the hot kernels (hipEvents recorded on the context's
 * stream around each launch), for benchmarks and roofline reports.
 * nut_ctx_kernel_time returns the total ms and launch count of one kernel kind
 * since the previous call (or since timing was enabled) and resets them. */
typedef enum {
  NUT_KERNEL_FILTER = 0,     /* filter scan + compaction          */
  NUT_KERNEL_AGGREGATE = 1,  /* fused filter/group-by/aggregate   */
  NUT_KERNEL_SORT = 2,       /* all radix-sort passes of one sort */
  NUT_KERNEL_JOIN = 3        /* hash join: build, count and write passes */
} nut_kernel_kind;
nut_status nut_ctx_enable_timing(nut_ctx *ctx, int enable);
nut_status nut_ctx_kernel_time(nut_ctx *ctx, int kind, double *total_ms, uint64_t *launches);
/* Algorithmic HBM bytes of the last nut_sort_i64[_desc] on this context (its levels
 * depend on the data: 8 B/key per histogram read, 16 B/key per scatter level, local sort
 * and copy) and the number of scatter levels it ran — the roofline numerator for sorts. */
nut_status nut_ctx_sort_stats(nut_ctx *ctx, uint64_t *bytes, uint32_t *levels);
/* The algorithm the last nut_groupby on this context took (parity tests and bench lines
 * name the path they checked): path = nut_groupby_path, levels = partition levels of a
 * partitioned path (0 otherwise), optimistic = how many of its leading levels ran without
 * a histogram pass (capped layout: 0, 1 or 2). */
typedef enum {
  NUT_GB_ONCHIP = 0,           /* streaming kernel, per-workgroup LDS tables (+ global table) */
  NUT_GB_PARTITIONED_DIRECT = 1, /* key-hash partition of the caller's columns, then LDS tables */
  NUT_GB_PARTITIONED_SPILL = 2,  /* WHERE / expressions staged first, then partitioned */
  NUT_GB_PARTITIONED_ORDERED = 3 /* nut_groupby_to_host: key-range partitions, ordered per partition, streamed to the host */
} nut_groupby_path;
nut_status nut_ctx_groupby_stats(nut_ctx *ctx, uint32_t *path, uint32_t *levels, uint32_t *optimistic);
/* Rows of the last nut_groupby_to_host on the ordered path (NUT_GB_PARTITIONED_ORDERED)
 * that did not fit their capped partition regions — a heavy key's excess, mostly — and
 * were aggregated from its overflow arenas and folded into the result (0: none); and, when
 * that call took the hashed path instead, why the ordered path declined. */
typedef enum {
  NUT_GB_DECLINE_NONE = 0,
  NUT_GB_DECLINE_SHAPE = 1,      /* not its shape: keys / aggregates / size / hint / alignment / key span */
  NUT_GB_DECLINE_CLUSTERED = 2,  /* the sample's distinct keys crowd some partitions (admission, before any work) */
  NUT_GB_DECLINE_ARENA = 3,      /* an overflow arena filled up */
  NUT_GB_DECLINE_CAPACITY = 4,   /* partition regions or tables do not fit their buffers */
  NUT_GB_DECLINE_TABLE = 5       /* a partition held more groups than its table */
} nut_gb_decline;
nut_status nut_ctx_groupby_overflow(nut_ctx *ctx, uint64_t *rows, uint32_t *declined);
/* The last ordered nut_groupby_to_host's heavy-key split (NUT_OPT_GB_HEAVY): how many keys
 * were aggregated in the streaming pass before the partition levels, and their rows. */
nut_status nut_ctx_groupby_heavy(nut_ctx *ctx, uint32_t *keys, uint64_t *rows);
/* The compiled Q1 kernel's launch shape on this context's device (NUT_OPT_PRIV_PROBE):
 * threads per workgroup and workgroups per CU the next launch takes, and the probe's best
 * kernel time per candidate shape {192 x 2, 128 x 3, 128 x 4} in ms (-1: not probed in
 * this process). */
nut_status nut_ctx_priv_shape(nut_ctx *ctx, int *threads, int *blocks_per_cu, double probe_ms[3]);
/* First-call latency of the probe: the call that runs it (the first compiled-Q1-shape
 * group-by of >= 2^27 rows on a device in the process) also times six full-size launches
 * of the kernel (2 rounds x 3 shapes) over the caller's input — at 1e9 rows ~45 ms, about
 * 7x that call's own kernel time — outside the kernel timers.  *ms = that wall time on this
 * context's device (0: not probed in this process).  NUT_OPT_PRIV_PROBE = 0 skips it. */
nut_status nut_ctx_priv_probe_cost(nut_ctx *ctx, double *ms);

/* Algorithm options of one context, for tuning A/B runs and tests that drive a path at
 * a size where the planner would not pick it.  The defaults are the product choice;
 * the library reads no environment variables.  Results never depend on them. */
typedef enum {
  NUT_OPT_GB_PARTITION = 0,    /* -1 auto (default), 0 never, 1 always (keyed group-bys) */
  NUT_OPT_GB_LEVELS = 1,       /* 0 auto (default), 1 or 2 partition levels */
  NUT_OPT_GB_OPTIMISTIC = 2,   /* 1 (default): first direct level without a histogram pass */
  NUT_OPT_GB_DIRECT = 3,       /* 1 (default): partition plain columns in place (no spill) */
  NUT_OPT_GB_CHUNKS = 4,       /* aggregation workgroups per CU over the partitions (8) */
  NUT_OPT_JOIN_REGION = 5,     /* 1 (default): LDS region build of large join tables */
  NUT_OPT_JOIN_PROBE_CFG = 6,  /* ordered probe tile shape 0..4 (0) */
  NUT_OPT_JOIN_ANY_CFG = 7,    /* unordered probe tile shape 0..4 (0) */
  NUT_OPT_GB_SEG_SLOTS = 8,    /* partition aggregation: LDS slots per hinted group, 1..8 (2) */
  NUT_OPT_GB_DENSE = 9,        /* 1 (default): whole partitions append their groups unhashed */
  NUT_OPT_GB_L1_BITS = 10,     /* digit bits of a capped second partition level, 6..8 (6) */
  NUT_OPT_TOPK = 11,           /* 1 (default): plans with ORDER BY ... LIMIT sort only nut_topk_positions' rows */
  NUT_OPT_GB_L0_BITS = 12,     /* digit bits of a capped first partition level, 6..8; 0 (default): 7 for one level up to 150 K groups, else 8; nut_groupby_to_host's ordered path: 7, with 14 - bits at level 1 */
  NUT_OPT_STREAM_BLOCKS = 13,  /* nut_stream_probe: workgroups per CU, 0 (default) = 8 */
  NUT_OPT_PRIV_BD = 14,        /* compiled Q1 kernel: threads per workgroup 128 / 192 / 256; 0 (default) = the probed shape (NUT_OPT_PRIV_PROBE), else 192 */
  NUT_OPT_PRIV_BLOCKS = 15,    /* compiled Q1 kernel: at most this many workgroups per CU; 0 (default) = the probed shape, else 2 */
  NUT_OPT_AGG_BLOCKS = 16,     /* shared-table streaming group-by: at most this many workgroups per CU; 0 (default) = as LDS allows */
  NUT_OPT_SEL_BLOCKS = 17,     /* expression scans (nut_select_rows): persistent workgroups per CU; 0 (default) = 8 */
  NUT_OPT_SORT_BD = 18,        /* sort, capped scatter levels: threads per workgroup 1024 (0, default) or 512 (two per CU) */
  NUT_OPT_GB_ORDERED = 19,     /* nut_groupby_to_host: the range-partitioned ordered path where it applies (1, default) or the hashed path + ordering (0) */
  NUT_OPT_PRIV_PROBE = 20,     /* 1 (default): the first compiled-Q1-shape group-by of >= 2^27 rows on a device times the kernel at 192 x 2, 128 x 3 and 128 x 4 threads x workgroups per CU over its whole input (two rounds, discarded) and keeps the fastest for that device, another shape than 192 x 2 only if >= 0.5 % faster (nut_ctx_priv_shape); 0: 192 x 2 */
  NUT_OPT_GB_HEAVY = 21,       /* nut_groupby_to_host, ordered path: 1 (default) = keys the sample sees often (>= 5 % of it together) are aggregated in one streaming pass and split off before the partition levels, and the levels' regions are laid out from exact per-cell counts of the rest; 2 = the split with capped levels (their overflow through the arenas); 0 = no split (the arenas take every excess) */
  NUT_OPT_JOIN_MATCH = 22,     /* ordered join probe (nut_join_*): 1 (default) = in two passes when no probe row can match two build rows (SEMI / ANTI, or unique build keys): the run walks in launch order into a 4-B-per-row match array, then the ordered write-out from it; 0 = one ordered pass */
  NUT_OPT_GB_L1_THREADS = 23,  /* nut_groupby_to_host, ordered path: the level-1 scatter's workgroup, 1024 (default: 16 Ki-record tiles) or 512 (8 Ki-record tiles in ~75 KB of LDS, so an aggregation workgroup of the previous chunk fits beside it on a CU) */
  NUT_OPT_AGG_SLOTS = 24,      /* streaming group-by, shared on-chip table: LDS slots per hinted group, 2..8 (4: load <= 1/4, a key almost always in its 4-slot home bucket); 2 halves the table so twice the workgroups fit a CU */
  NUT_OPT_GB_L1_SPARE = 25,    /* nut_groupby_to_host, ordered path: CUs the level-1 scatter of chunks after the first leaves free for the previous chunk's aggregation, 0..128 (32: G = 1e7 step 20.6-20.8 vs 21.4 ms at 0, same box; 64: 20.5 vs 20.9) */
  NUT_OPT_COUNT = 26
} nut_option;
nut_status nut_ctx_set_option(nut_ctx *ctx, int option, int64_t value);
nut_status nut_ctx_get_option(nut_ctx *ctx, int option, int64_t *value);

/* ------------------------------------------------------------------------
 * Synthetic columns (bench / tests): counter-based splitmix64 generator,
 * bit-identical to oracle/oracle.c orc_gen_column and numpy
 * (tests/golden/make_golden.py).  u = mix64(seed + (row0+i+1) * 0x9E3779B97F4A7C15).
 * ------------------------------------------------------------------------ */
typedef enum {
  NUT_GEN_U62 = 0,       /* int64: u >> 2                         */
  NUT_GEN_FULL_I64 = 1,  /* int64: u                              */
  NUT_GEN_POOL_KEY = 2,  /* int64: mix64((u % a) ^ 0x5DEECE66D2545F49) — a distinct keys */
  NUT_GEN_DYADIC = 3,    /* f64: (u >> 44) / 64                   */
  NUT_GEN_UNIT_F64 = 4,  /* f64: (u >> 11) * 2^-53                */
  NUT_GEN_RANGE_I64 = 5, /* int64: a + u % b                      */
  NUT_GEN_RANGE_F64 = 6, /* f64: (double)(a + u % b) / c          */
  NUT_GEN_SKEW_KEY = 7   /* int64: mix64(((u % a) >> ((mix64(u) >> 59) * 3 >> 2)) ^ 0x5DEECE66D2545F49) —
                            a log-uniform (Zipf-like, exponent ~1) draw of a distinct keys: pool index 0
                            takes ~3 %, index i ~ 1 / i of the rows */
} nut_gen_kind;

nut_status nut_gen_column(nut_ctx *ctx, int kind, uint64_t seed, int64_t a, int64_t b,
                          double c, uint64_t row0, uint64_t n, void *out);

/* Copy-floor probe ("the fraction of a measured in-build device-copy
 * kernel's bandwidth"): streams read_bytes from src with 16-B non-temporal loads and writes
 * write_bytes (<= read_bytes) of them to dst with non-temporal stores, interleaved at the
 * same read:write ratio as a scan that keeps that fraction of its input.  Both sizes are
 * multiples of 16, the buffers 16-B aligned, dst holds write_bytes + 1 KiB.  Runs `reps`
 * launches at 2, 4 and 8 workgroups of 256 threads per CU (or NUT_OPT_STREAM_BLOCKS) on
 * the context's stream and returns the fastest one's device time (hipEvents) in *best_ms. */
nut_status nut_stream_probe(nut_ctx *ctx, const void *src, uint64_t read_bytes, void *dst,
                            uint64_t write_bytes, int reps, double *best_ms);

/* ------------------------------------------------------------------------
 * Filter scan + selection-vector compaction (BASELINE config 2)
 *   SELECT col FROM t WHERE col <cmp> k
 * Lowered from WhereClause{BinaryOp{Identifier, op, Literal::Integer}}
 * (src/parser/ast/query.rs:68-72, expr.rs:25-30, item.rs:89-101).
 * Output keeps row order.  `out` must hold n elements (worst case).
 * ------------------------------------------------------------------------ */
typedef enum {
  NUT_LT = 0, NUT_LE = 1, NUT_GT = 2, NUT_GE = 3, NUT_EQ = 4, NUT_NE = 5,
  NUT_IN = 6, NUT_NOT_IN = 7  /* set membership: nut_agg_spec predicates only */
} nut_cmp;

nut_status nut_filter_i64(nut_ctx *ctx, const int64_t *col, uint64_t n, int cmp, int64_t k,
                          int64_t *out, uint64_t *out_n_host);
/* as above; the count is written to device memory out_n_dev, no synchronisation */
nut_status nut_filter_i64_async(nut_ctx *ctx, const int64_t *col, uint64_t n, int cmp,
                                int64_t k, int64_t *out, uint64_t *out_n_dev);

/* ------------------------------------------------------------------------
 * Fused filter -> hash group-by -> aggregate (BASELINE configs 3 and 4)
 *   SELECT k1[,k2], agg(expr)... FROM t WHERE p1 AND p2 ... GROUP BY k1[,k2]
 * Lowered from WhereClause (AND-chain of `col op literal`), GroupByClause.keys
 * (identifiers) and the SELECT list's FnCall{Others("sum"|"count"|"min"|"max")}.
 * ------------------------------------------------------------------------ */
typedef enum { NUT_T_I64 = 0, NUT_T_F64 = 1, NUT_T_STR = 2 /* result columns of typed tables only */ } nut_type;
typedef enum { NUT_AGG_SUM = 0, NUT_AGG_COUNT = 1, NUT_AGG_MIN = 2, NUT_AGG_MAX = 3 } nut_agg_op;
typedef enum {
  NUT_EX_COL = 0,       /* v[a]                      (i64 or f64 column) */
  NUT_EX_MUL = 1,       /* v[a] * v[b]               (f64)               */
  NUT_EX_ADD = 2,       /* v[a] + v[b]                                   */
  NUT_EX_SUB = 3,       /* v[a] - v[b]                                   */
  NUT_EX_MUL_1M = 4,    /* v[a] * (1 - v[b])         (TPC-H disc_price)  */
  NUT_EX_MUL_1M_1P = 5  /* v[a] * (1 - v[b]) * (1 + v[c])  (charge)      */
} nut_expr;

#define NUT_MAX_KEYS 2
#define NUT_MAX_PRED 6
#define NUT_MAX_VALS 4
#define NUT_MAX_AGGS 8
#define NUT_MAX_SET 16
#define NUT_MAX_PROG_COLS 16
#define NUT_MAX_PROG_NODES 256

/* Expression programs: postfix (RPN) node arrays.  Every node pops its operands and
 * pushes one value of type int64, float64 or bool (nut_prog_type gives the result).
 *   COL      push prog_col[arg]
 *   I64/F64  push the constant v (F64: the double's bits)
 *   arithmetic  i64 (+ - *) wraps; any f64 operand makes the op f64; DIV is always
 *            f64 (int operands converted); MOD/INTDIV on ints truncate toward zero and
 *            fail the query on a zero divisor (INT64_MIN % -1 = 0, INT64_MIN div -1
 *            wraps); MOD on f64 is fmod
 *   compare  bool; an int compared with an f64 converts the int to f64
 *   AND OR XOR NOT  bool operands (ints: non-zero = true), no short circuit
 *   BITAND BITOR BITXOR BITNOT SHL SHR  ints; shift counts outside [0, 63] give 0
 *            (SHR of a negative value: -1); SHR is arithmetic
 *   IF       pops cond, then, else: the chosen branch (only its errors count)
 *   ABS, TO_F64  one operand; bool operands count as int 0/1 in arithmetic
 *   LOOKUP   one int operand x; v = device address of a byte table, arg = its length:
 *            bool table[x] != 0 for 0 <= x < arg, else false (dictionary predicates such
 *            as LIKE over dictionary codes; the table must outlive the call)
 *   MAP      one int operand x; v = device address of an int64 table, arg = its length:
 *            int table[x] for 0 <= x < arg, else -1 (dictionary functions such as
 *            substring over dictionary codes: code -> the result string's code)
 *   DATEPART one int operand d = days since 1970-01-01 (proleptic Gregorian), int result
 *            by arg (nut_date_part): year, month 1-12, day of month, quarter 1-4, day of
 *            week (Monday = 1 .. Sunday = 7), day of year 1-366, year * 100 + month,
 *            year * 10000 + month * 100 + day (toYYYYMM / toYYYYMMDD); d is first clamped to
 *            [-2^40, 2^40] (beyond any real date), so every d has one defined result. */
typedef enum {
  NUT_P_COL = 0, NUT_P_I64 = 1, NUT_P_F64 = 2,
  NUT_P_ADD = 3, NUT_P_SUB = 4, NUT_P_MUL = 5, NUT_P_DIV = 6, NUT_P_MOD = 7, NUT_P_INTDIV = 8,
  NUT_P_LT = 9, NUT_P_LE = 10, NUT_P_GT = 11, NUT_P_GE = 12, NUT_P_EQ = 13, NUT_P_NE = 14,
  NUT_P_AND = 15, NUT_P_OR = 16, NUT_P_XOR = 17, NUT_P_NOT = 18,
  NUT_P_BITAND = 19, NUT_P_BITOR = 20, NUT_P_BITXOR = 21, NUT_P_BITNOT = 22,
  NUT_P_SHL = 23, NUT_P_SHR = 24,
  NUT_P_IF = 25, NUT_P_ABS = 26, NUT_P_TO_F64 = 27, NUT_P_LOOKUP = 28, NUT_P_DATEPART = 29,
  NUT_P_MAP = 30
} nut_prog_op;
typedef enum {
  NUT_DP_YEAR = 0, NUT_DP_MONTH = 1, NUT_DP_DAY = 2, NUT_DP_QUARTER = 3, NUT_DP_WEEKDAY = 4, NUT_DP_YEARDAY = 5,
  NUT_DP_YYYYMM = 6, NUT_DP_YYYYMMDD = 7
} nut_date_part;
typedef enum { NUT_PT_I64 = 0, NUT_PT_F64 = 1, NUT_PT_BOOL = 2 } nut_prog_value_type;
typedef struct {
  int32_t op;   /* nut_prog_op */
  int32_t arg;  /* NUT_P_COL: column index; NUT_P_LOOKUP / MAP: table length; NUT_P_DATEPART: part */
  int64_t v;    /* NUT_P_I64 / NUT_P_F64 constant; NUT_P_LOOKUP / MAP: table address */
} nut_prog_node;
typedef struct {
  int32_t n;                  /* 0..NUT_MAX_PROG_NODES */
  const nut_prog_node *node;  /* host memory */
} nut_prog;
/* Type-check a program against column types; *type = nut_prog_value_type of the
 * result.  NUT_ERR_INVALID_ARG (message in nut_last_error) if it is malformed. */
nut_status nut_prog_type(const nut_prog *prog, const int32_t *col_types, int ncols, int32_t *type);

typedef struct {
  uint64_t n;                          /* rows */
  int32_t nkeys;                       /* 1..2 int64 key columns; 0 = global aggregate
                                          (no GROUP BY: at most one group, key word 0) */
  const int64_t *keys[NUT_MAX_KEYS];
  int32_t npred;                       /* conjunction of npred terms (0 = no WHERE) */
  const void *pred_col[NUT_MAX_PRED];
  int32_t pred_type[NUT_MAX_PRED];     /* nut_type */
  int32_t pred_op[NUT_MAX_PRED];       /* nut_cmp */
  int64_t pred_i64[NUT_MAX_PRED];      /* constant when pred_type == NUT_T_I64 */
  double pred_f64[NUT_MAX_PRED];       /* constant when pred_type == NUT_T_F64 */
  int32_t nvals;                       /* value columns referenced by expressions */
  const void *val_col[NUT_MAX_VALS];
  int32_t val_type[NUT_MAX_VALS];      /* nut_type; expressions other than COL need f64 */
  int32_t naggs;
  int32_t agg_op[NUT_MAX_AGGS];        /* nut_agg_op */
  int32_t agg_expr[NUT_MAX_AGGS];      /* nut_expr (ignored for COUNT) */
  int32_t agg_arg[NUT_MAX_AGGS][3];    /* value-column indices of the expression */
  /* pred_op NUT_IN / NUT_NOT_IN: `col [NOT] IN (set)` with pred_nset[t] in 1..16 values
   * (an f64 column's values as the doubles' bits) */
  int32_t pred_nset[NUT_MAX_PRED];
  int64_t pred_set[NUT_MAX_PRED][NUT_MAX_SET];
  /* Expression mode (prog_mode = 1): WHERE and every aggregate
   * argument are expression programs over prog_col[], compiled at run time into the
   * same streaming kernel.  pred_*, val_* and agg_expr/agg_arg must then be unused
   * (npred = nvals = 0).  Types follow nut_prog_type. */
  int32_t prog_mode;
  int32_t nprog_cols;
  const void *prog_col[NUT_MAX_PROG_COLS];
  int32_t prog_col_type[NUT_MAX_PROG_COLS]; /* nut_type */
  nut_prog where;                           /* n = 0: every row */
  nut_prog agg_val[NUT_MAX_AGGS];           /* argument of each non-COUNT aggregate */
  nut_prog agg_mask[NUT_MAX_AGGS];          /* n = 0: every row; else the aggregate takes
                                               only rows where it is true (SQL NULL
                                               arguments of CASE without ELSE) */
  /* Expression mode: key j (j < nkeys) is the value of key_prog[j] when its n > 0 (an
   * int64 or bool program; keys[j] is then unused and may be NULL), else keys[j].
   * Computed keys (getYear(d), a % 10) and packed key tuples: SQL plans pack up to 8
   * GROUP BY keys into two words this way. */
  nut_prog key_prog[NUT_MAX_KEYS];
} nut_agg_spec;

/* Result word per aggregate: f64 bits for SUM/MIN/MAX of an f64 expression,
 * int64 for COUNT and for SUM/MIN/MAX of an int64 column (SUM wraps).
 * MIN/MAX order f64 by the IEEE total order (-0 < +0).  Expression mode: f64 bits
 * when the program's type is f64, else int64 (bool = 0/1); an aggregate whose mask
 * took no row of a group holds its identity (SUM/COUNT 0, MIN/MAX the type's
 * largest/smallest value; f64: 0x7FFF... / 0xFFFF..., the NaN patterns at the
 * two ends of the IEEE total order).
 *
 * group_hint: expected number of groups (0 = unknown).  It sizes the on-chip
 * table; a wrong hint costs speed, never correctness. */
nut_status nut_groupby(nut_ctx *ctx, const nut_agg_spec *spec, uint64_t group_hint,
                       nut_groups **out);
/* Aggregate more rows (same spec shape) into an existing result, e.g. to merge
 * the partial groups received from other ranks (NUT_AGG_COUNT partials are merged
 * with NUT_AGG_SUM over an int64 column). */
nut_status nut_groupby_accumulate(nut_ctx *ctx, const nut_agg_spec *spec, nut_groups *acc);

/* Expression mode: the HIP source of the query-specific kernel shape (generated from
 * the programs; constants travel as kernel arguments, so queries that differ only in
 * constants share one compiled kernel), and a compile-only check of it (hipRTC,
 * gfx950; no device needed).  The compile log of a failure is in nut_last_error. */
nut_status nut_groupby_jit_source(const nut_agg_spec *spec, char *buf, size_t cap, size_t *len);
nut_status nut_groupby_jit_compile(const nut_agg_spec *spec);

nut_status nut_groups_size(nut_groups *g, uint64_t *n_groups);
/* Copy to host sorted ascending by key tuple.  keys[g*nkeys+j], aggs[g*naggs+a].
 * cap = capacity in groups; NUT_ERR_CAPACITY if too small. */
nut_status nut_groups_to_host(nut_groups *g, int64_t *keys, uint64_t *aggs, uint64_t cap);
/* Dense device copy, column-major: out_dev[w * n + g], w = 0..nkeys-1 keys then
 * naggs aggregate words; needs (nkeys+naggs)*n words.  Unordered. */
nut_status nut_groups_to_device(nut_groups *g, uint64_t *out_dev, uint64_t cap);
/* Partition the groups by owner rank = mix64(key tuple) % nparts for the
 * multi-GPU exchange: segment p (counts_host[p] groups) is stored column-major
 * like nut_groups_to_device at word offset (nkeys+naggs) * sum_{q<p} counts[q]. */
nut_status nut_groups_partition(nut_groups *g, int nparts, uint64_t *out_dev, uint64_t cap,
                                uint64_t *counts_host);
void nut_groups_free(nut_groups *g);
/* nut_groupby + nut_groups_to_host + nut_groups_free in one call: the groups sorted
 * ascending by key into keys[g*nkeys+j] / aggs[g*naggs+a] (cap groups of room), their
 * number in *n_out (also on NUT_ERR_CAPACITY: the room needed).  For one plain key column
 * and plain-column aggregates over >= 2^24 rows with group_hint >= ~1.6e6 and page-locked
 * outputs, the groups are partitioned by key range so that they come out ordered without
 * a sort, and the result crosses to the host in chunks while the rest is computed
 * (nut_ctx_groupby_stats: NUT_GB_PARTITIONED_ORDERED); every other case runs the three
 * calls.  The results are the same either way. */
nut_status nut_groupby_to_host(nut_ctx *ctx, const nut_agg_spec *spec, uint64_t group_hint, int64_t *keys,
                               uint64_t *aggs, uint64_t cap, uint64_t *n_out);

/* Convenience forms named in SURVEY.md §8(b). */
#define NUT_AGGMASK_SUM 1u
#define NUT_AGGMASK_COUNT 2u
#define NUT_AGGMASK_MIN 4u
#define NUT_AGGMASK_MAX 8u
/* SELECT key, [sum(val)], [count(*)], [min(val)], [max(val)] FROM t GROUP BY key */
nut_status nut_groupby_i64_f64(nut_ctx *ctx, const int64_t *key, const double *val,
                               uint64_t n, uint32_t agg_mask, uint64_t group_hint,
                               nut_groups **out);
/* TPC-H Q1 shape: SELECT returnflag, linestatus, sum(qty), sum(price),
 *   sum(price*(1-disc)), count(*) FROM lineitem WHERE shipdate <= date_k
 *   GROUP BY returnflag, linestatus */
nut_status nut_q1(nut_ctx *ctx, const int64_t *shipdate, const int64_t *returnflag,
                  const int64_t *linestatus, const double *qty, const double *price,
                  const double *disc, uint64_t n, int64_t date_k, nut_groups **out);

/* ------------------------------------------------------------------------
 * Sort (BASELINE config 5): SELECT k FROM t ORDER BY k  (ascending int64)
 * Lowered from OrderByClause (src/parser/ast/query.rs:86-90).  in and out may
 * not alias.  Scratch is owned by the context.
 * ------------------------------------------------------------------------ */
nut_status nut_sort_i64(nut_ctx *ctx, const int64_t *in, int64_t *out, uint64_t n);
/* ORDER BY k DESC (the same passes with the key order complemented; no extra pass) */
nut_status nut_sort_i64_desc(nut_ctx *ctx, const int64_t *in, int64_t *out, uint64_t n);
/* ORDER BY with projected columns (OrderByClause.keys, query.rs:86-90): a STABLE sort of
 * (key, payload) pairs that returns the payload in key order — vals_out[i] = the payload
 * of the i-th smallest key (DESC: largest), ties in input order.  keys: n int64
 * (key_type NUT_T_I64) or float64 (NUT_T_F64, IEEE total order: -NaN < -inf < ... < -0 <
 * +0 < ... < +inf < NaN) values; vals: n int64 payloads, or NULL for the row ids 0..n-1.
 * Several ORDER BY keys: sort by the last key first and feed each result as the next
 * call's payload (LSD order, the sort is stable).  vals and vals_out may not alias. */
nut_status nut_sort_pairs(nut_ctx *ctx, const void *keys, int key_type, int desc, const int64_t *vals,
                          int64_t *vals_out, uint64_t n);
/* ORDER BY ... LIMIT k (LimitClause, query.rs:92-98) without sorting every row: the
 * positions, ascending, of every key ordered at or before the k-th smallest (desc:
 * largest) of n keys (key_type / order as nut_sort_pairs) — at least k of them, every tie
 * of the k-th key and a few more included, so a stable sort of just these rows yields the
 * first k rows of the full sort.  *count_host = their number; NUT_ERR_CAPACITY (no
 * message) if it exceeds cap (positions untouched).  Radix select: 12-bit digit
 * histograms, 8 B/key per level (usually one), + 8 B/key to collect. */
nut_status nut_topk_positions(nut_ctx *ctx, const void *keys, int key_type, int desc, uint64_t n, uint64_t k,
                              int64_t *positions, uint64_t cap, uint64_t *count_host);
/* Stable partition of int64 keys into nsplit+1 buckets, bucket(k) = #{i : splitters[i] <= k}
 * (splitters_host ascending, 0 <= nsplit < 64).  Bucket b is written to out at offset
 * sum_{c<b} counts_host[c]; counts_host receives nsplit+1 counts.  The local step of the
 * multi-GPU sample sort: partition by splitters, all-to-all,
 * local nut_sort_i64. */
nut_status nut_partition_i64(nut_ctx *ctx, const int64_t *in, uint64_t n, const int64_t *splitters_host,
                             int nsplit, int64_t *out, uint64_t *counts_host);

/* ------------------------------------------------------------------------
 * Hash join: equi-join on one int64 key, lowered from
 * JoinClause{typ, source, condition: On(a = b)} (src/parser/ast/query.rs:55-66,
 * 100-117).  `build` is the joined table (the JoinClause source), `probe` the
 * FROM table.  The result is a join index: pairs (probe row, build row) ordered
 * by probe row; the build rows of one probe row are in unspecified order.
 *   NUT_JOIN_INNER  every matching pair
 *   NUT_JOIN_LEFT   LEFT OUTER: as INNER, plus (p, -1) for probe rows without a match
 *   NUT_JOIN_SEMI   LEFT SEMI: (p, -1) once per probe row with >= 1 match
 *   NUT_JOIN_ANTI   LEFT ANTI: (p, -1) for probe rows without a match
 * (RIGHT variants are the LEFT ones with the tables swapped.)  Keys are device
 * pointers; the index arrays live in HBM, owned by the nut_join.
 * ------------------------------------------------------------------------ */
typedef enum { NUT_JOIN_INNER = 0, NUT_JOIN_LEFT = 1, NUT_JOIN_SEMI = 2, NUT_JOIN_ANTI = 3 } nut_join_type;
/* OR-ed into join_type: the pairs may come out in any order (aggregates over a join need
 * none) — one unordered probe pass with no tile ordering */
#define NUT_JOIN_ANY_ORDER 0x100
typedef struct nut_join nut_join;
/* builds the table and counts the pairs (the key arrays must stay valid until
 * nut_join_write); *npairs receives the result length */
nut_status nut_join_i64(nut_ctx *ctx, const int64_t *build, uint64_t nbuild, const int64_t *probe, uint64_t nprobe,
                        int join_type, nut_join **out, uint64_t *npairs);
/* writes the npairs pairs into caller-owned device arrays */
nut_status nut_join_write(nut_join *j, int64_t *probe_idx, int64_t *build_idx);
void nut_join_free(nut_join *j);
/* one-pass form: builds the table and writes the pairs straight into caller-owned device
 * arrays of `cap` entries; *npairs = the result length.  NUT_ERR_CAPACITY when it exceeds
 * cap (no pair is valid then: call again with cap >= *npairs).  cap = nprobe always
 * suffices for LEFT SEMI / ANTI, and for INNER / LEFT when the build keys are unique. */
nut_status nut_join_i64_into(nut_ctx *ctx, const int64_t *build, uint64_t nbuild, const int64_t *probe,
                             uint64_t nprobe, int join_type, int64_t *probe_idx, int64_t *build_idx, uint64_t cap,
                             uint64_t *npairs);
/* Expression-mode scan + compaction: the row ids (ascending) of the
 * rows where s->where holds — any program over s->prog_col, compiled for the query like
 * the expression-mode group-by.  Reads s->n, s->where and the program columns only (keys
 * and aggregates are ignored).  out_rows holds s->n entries (worst case); *count_host =
 * rows selected.  Carry any column through the ids with nut_gather_u64. */
nut_status nut_select_rows(nut_ctx *ctx, const nut_agg_spec *s, int64_t *out_rows, uint64_t *count_host);
/* compile the scan kernel of nut_select_rows for this spec (hipRTC; no GPU needed) */
nut_status nut_select_jit_compile(const nut_agg_spec *s);
/* Computed projections (SELECT a * b, CASE ..., toYYYYMMDD(d) FROM t):
 * for i < m, out[a][i] = program s->agg_val[a] (a < s->naggs, agg_op ignored) evaluated
 * at row rows[i] of the program columns (rows NULL: row i, m <= s->n), as 8-byte words
 * (int64, or float64 bits when nut_prog_type says F64); valid[a][i] = 1 where the mask
 * program s->agg_mask[a] holds (always without one), else 0 with out[a][i] = 0 — a SQL
 * NULL.  valid NULL or valid[a] NULL: not written.  Row ids must index the program
 * columns (nut_select_rows output does).  Division by zero: NUT_ERR_INVALID_ARG. */
nut_status nut_eval_rows(nut_ctx *ctx, const nut_agg_spec *s, const int64_t *rows, uint64_t m, uint64_t *const *out,
                         uint8_t *const *valid);
nut_status nut_eval_jit_compile(const nut_agg_spec *s);
/* The multi-GPU join's exchange step: rows go to part (owner_hash(key) >> 56) * nparts / 256
 * (owner_hash = the group-by's; host restatement nutdb_amd/dist.py join_owner); out_keys /
 * out_rows (row0 + row index) hold the parts one after another in part order, rows
 * unordered within a part; counts_host[nparts] receives the part sizes.  nparts in [1, 256]. */
nut_status nut_hash_partition_i64(nut_ctx *ctx, const int64_t *keys, uint64_t n, int nparts, int64_t row0,
                                  int64_t *out_keys, int64_t *out_rows, uint64_t *counts_host);
/* out[i] = src[idx[i]] (8-byte words), or `null_bits` where idx[i] < 0: carries any
 * int64 / f64 column through a join index.  out may be idx itself (in place); it must
 * not overlap src. */
nut_status nut_gather_u64(nut_ctx *ctx, const uint64_t *src, const int64_t *idx, uint64_t n, uint64_t null_bits,
                          uint64_t *out);

/* ========================================================================
 * Multi-GPU execution over RCCL (SURVEY.md §8(b) nut_dist_*, §8(e)).
 * A nut_dist is a group of P ranks, one GPU each; this process drives `nlocal` of them
 * (its "local members", global ranks first_rank .. first_rank+nlocal-1), each with its
 * own nut_ctx and RCCL communicator.  Three ways to form one:
 *   nut_dist_create        one process drives ndev GPUs (ncclCommInitAll); the
 *                          nut_dist_* calls run one host thread per device
 *   nut_dist_create_rank   one process per GPU (MPI / torchrun style): rank 0 makes an
 *                          id with nut_dist_unique_id, the host shares its
 *                          NUT_DIST_ID_BYTES bytes with every rank (ncclCommInitRank)
 *   nut_dist_create_virtual  P ranks on ONE device whose exchanges are device copies
 *                          instead of RCCL: the same partition / exchange / merge code
 *                          with P > 1 on a single GPU (tests)
 * Every nut_dist_* call is collective: each process calls it with arrays of nlocal
 * entries (entry l = local member l's shard; device pointers on that member's device).
 * Rows are sharded by rank; the exchange is one all-to-all of counts (an all-gather,
 * which also carries every rank's status so a failure on one rank fails the call on
 * all of them instead of hanging the others) and one ncclAllToAllv of records.
 * ======================================================================== */
typedef struct nut_dist nut_dist;
#define NUT_DIST_ID_BYTES 128
nut_status nut_dist_create(int ndev, const int *devs, nut_dist **out);
nut_status nut_dist_unique_id(void *id);
nut_status nut_dist_create_rank(int nranks, int rank, const void *id, int device, nut_dist **out);
nut_status nut_dist_create_virtual(int nranks, int device, nut_dist **out);
nut_status nut_dist_info(const nut_dist *d, int *nranks, int *nlocal, int *first_rank);
/* context of local member l (timing, synthetic columns, single-GPU calls on its shard) */
nut_ctx *nut_dist_ctx(nut_dist *d, int local);
/* Collective like every nut_dist call.  Free the nut_groups a nut_dist_groupby returned
 * first: they live on a member's context, which this destroys. */
void nut_dist_destroy(nut_dist *d);

/* Group-by across ranks (configs 3, 4): local pre-aggregation of specs[l] on member l ->
 * partial groups partitioned by owner = mix64(key tuple) % P -> ncclAllToAllv -> each
 * owner merges what it received (SUM / COUNT add, MIN / MAX re-min/max) -> the owners'
 * groups are gathered on rank 0.  out[l] = the global result on the member holding
 * rank 0, NULL on every other member.  Every rank's spec has the same shape. */
nut_status nut_dist_groupby(nut_dist *d, const nut_agg_spec *specs, uint64_t group_hint, nut_groups **out);
/* ORDER BY k across ranks (config 5), sample sort: 4096 strided samples per rank ->
 * all-gather -> P-1 splitters at the pooled sample's quantiles -> nut_partition_i64 ->
 * ncclAllToAllv of keys -> local nut_sort_i64.  Member l ends with out_n[l] keys at
 * out[l] (device memory owned by the member, valid until its next nut_dist_* call):
 * the r-th key range of the global order, so the ranks' outputs concatenated in rank
 * order are sorted.  Keys equal to a splitter go to the higher rank.  P <= 64. */
nut_status nut_dist_sort_i64(nut_dist *d, const int64_t *const *in, const uint64_t *n, const int64_t **out,
                             uint64_t *out_n);
/* SELECT col FROM t WHERE col <cmp> k over row shards (config 2): no data exchange;
 * out_n[l] = rows member l selected (into its caller-owned out[l], n[l] entries),
 * out_offset[l] = their position in the global result (the rank-ordered concatenation). */
nut_status nut_dist_filter_i64(nut_dist *d, const int64_t *const *col, const uint64_t *n, int cmp, int64_t k,
                               int64_t *const *out, uint64_t *out_n, uint64_t *out_offset);
/* Hash join across ranks (§8(f) 4): both sides hash-partitioned by key owner
 * (nut_hash_partition_i64), one ncclAllToAllv of (key, global row) records per side, a
 * local nut_join_i64 on every rank.  Global row ids: build_row0[l] / probe_row0[l] = the
 * global index of member l's first row.  Member l ends with npairs[l] pairs of GLOBAL
 * (probe row, build row) at probe_idx[l] / build_idx[l] (member-owned, valid until its
 * next nut_dist_* call; -1 = no build row), nut_join_i64 semantics per key. */
nut_status nut_dist_join_i64(nut_dist *d, const int64_t *const *build, const uint64_t *nbuild, const int64_t *build_row0,
                             const int64_t *const *probe, const uint64_t *nprobe, const int64_t *probe_row0,
                             int join_type, const int64_t **probe_idx, const int64_t **build_idx, uint64_t *npairs);

/* ========================================================================
 * SQL front end (CPU) — restatement of the reference's only public API,
 *   nutdb::parser::Parser::parse(&str) -> Result<Statement, ParseError>
 *   (src/lib.rs:3-4, src/parser/mod.rs:26-29)
 * Accept/reject behaviour, error texts (src/parser/error.rs:8-57) and constant
 * folding (src/parser/simplify.rs) follow the reference, quirks included
 * (SURVEY.md §8(a) A8).  These entry points never touch a GPU.
 * Errors: NUT_ERR_PARSE with nut_last_error() = the ParseError Display text
 * ("Lex Error: ..." / "Syntax Error: ...").
 * ======================================================================== */
typedef struct nut_stmt nut_stmt;

/* Statement variants, in the order of src/parser/ast/mod.rs:13-24 */
typedef enum {
  NUT_STMT_SELECT = 0, NUT_STMT_INSERT = 1, NUT_STMT_EXPLAIN = 2, NUT_STMT_ALTER = 3,
  NUT_STMT_CREATE = 4, NUT_STMT_DESCRIBE = 5, NUT_STMT_DROP = 6, NUT_STMT_TRUNCATE = 7,
  NUT_STMT_OPTIMIZE = 8, NUT_STMT_SET = 9
} nut_stmt_kind;

/* Parser::parse.  `sql` need not be NUL-terminated; it must be valid UTF-8 (the
 * reference takes &str).  The statement keeps its own copy of the text. */
nut_status nut_sql_parse(const char *sql, size_t len, nut_stmt **out);
int nut_stmt_kind_of(const nut_stmt *stmt);
/* S-expression of the tree (grammar in nutdb_amd/csrc/sql_dump.cpp).  Writes at
 * most cap-1 bytes + NUL; *len (optional) = full length, so a too-small buffer
 * returns NUT_ERR_CAPACITY with the size needed. */
nut_status nut_stmt_dump(const nut_stmt *stmt, char *buf, size_t cap, size_t *len);
void nut_stmt_free(nut_stmt *stmt);

/* Tokenizer::next_token (src/parser/tokenizer/mod.rs:66-112) until EOF, whitespace
 * and comment tokens included.  types[i] = TokenType index (token.rs:5-91 order,
 * KeywordOrIdentifier = 0 ... EOF = 39); spans[2i], spans[2i+1] = byte offsets.
 * *ntok = tokens produced (EOF included).  NUT_ERR_PARSE on a lexical error
 * (the tokens before it are still written), NUT_ERR_CAPACITY if cap is short. */
nut_status nut_sql_tokenize(const char *sql, size_t len, int32_t *types, uint64_t *spans, size_t cap,
                            size_t *ntok);
/* unescape_{single,double}_quoted_string (src/parser/literal.rs:36-103); quote is
 * '\'' or '"'.  Output is not NUL-terminated; *out_len = bytes. */
nut_status nut_sql_unescape(const char *s, size_t len, int quote, char *out, size_t cap, size_t *out_len);

/* ========================================================================
 * Plan lowering and execution.  A plan is lowered from the
 * statement tree — QueryBody.r#where / group_by / columns / order_by / limit
 * (src/parser/ast/query.rs:21-35) — and executed on the kernels above with the
 * plan's column names bound to device columns at execute time.
 *   FILTER : SELECT c FROM t [WHERE c <cmp> const]          [LIMIT]
 *   GROUPBY: SELECT k.., agg(expr).. FROM t [WHERE conj] GROUP BY k1[,k2]
 *            [ORDER BY outputs] [LIMIT]; agg in sum/count/min/max/avg
 *   SORT   : SELECT c FROM t [WHERE c <cmp> const] ORDER BY c [DESC] [LIMIT]
 * Constants may be integer/float literals, toDate('YYYY-MM-DD') and date +/-
 * interval n day|month|year (days since 1970-01-01).
 * Lowering failures return NUT_ERR_PLAN with a message naming the construct.
 * ======================================================================== */
typedef struct nut_plan nut_plan;
typedef struct nut_result nut_result;

typedef enum { NUT_PLAN_FILTER = 0, NUT_PLAN_GROUPBY = 1, NUT_PLAN_SORT = 2 } nut_plan_kind;

typedef struct {
  const char *name;   /* column name as written in the SQL (ASCII case-insensitive match) */
  const void *data;   /* device pointer, nrows elements (host pointer with NUT_COL_HOST) */
  int32_t type;       /* nut_type, optionally | NUT_COL_HOST */
} nut_column;
/* OR-ed into nut_column.type: `data` is host memory (pageable or page-locked).  The
 * nut_plan_execute* calls copy such a column into HBM on the context's stream (8 B x nrows
 * over PCIe) before running the plan and free the copy before they return; the caller
 * keeps ownership.  Device-resident columns are read in place. */
#define NUT_COL_HOST 0x100

nut_status nut_sql_plan(const char *sql, size_t len, nut_plan **out);
int nut_plan_kind_of(const nut_plan *plan);
/* JSON description of the plan (columns, predicates, aggregates, outputs); same
 * buffer convention as nut_stmt_dump */
nut_status nut_plan_describe(const nut_plan *plan, char *buf, size_t cap, size_t *len);
/* The executor route a single-table plan takes over columns of the given names and types
 * (`data` may be NULL: host only, no device, nothing runs) — "fused-filter", "fused-sort",
 * "expr-filter", "expr-sort", "expr-sort-f64-order" (float64 bits sorted as int64 words in
 * the IEEE total order), "rowid-scan", "rerun-expression -> …", "fused-groupby",
 * "expr-groupby", "packed-groupby" — or the NUT_ERR_PLAN nut_plan_execute would return.
 * A test hook for the routing; same buffer convention as nut_stmt_dump. */
nut_status nut_plan_route(const nut_plan *plan, const nut_column *cols, int ncols, char *buf, size_t cap,
                          size_t *len);
void nut_plan_free(nut_plan *plan);

/* Compile an expression-mode plan's kernel now (hipRTC; no device needed) so the first
 * nut_plan_execute does not pay for it.  Columns bind by name like execute; only their
 * types matter (data may be NULL).  A no-op for plans on the precompiled kernels. */
nut_status nut_plan_prepare(const nut_plan *plan, const nut_column *cols, int ncols);
/* Execute on nrows rows of the bound columns (every column the plan names must be
 * bound).  group_hint as for nut_groupby.  Synchronous.  A plan with uncorrelated scalar
 * subqueries (`x > (SELECT avg(x) FROM t ...)`, describe: "subqueries") runs each of them
 * first over the same columns (nut_plan_execute / nut_table_execute only; the multi-table
 * entry points reject such plans with NUT_ERR_UNSUPPORTED). */
nut_status nut_plan_execute(nut_ctx *ctx, const nut_plan *plan, const nut_column *cols, int ncols,
                            uint64_t nrows, uint64_t group_hint, nut_result **out);
/* A plan with a JOIN: `left` = the FROM table (lrows rows), `right` = the JOIN source.
 * Every plan column is bound in exactly one of them (names unique across the two).
 * The ON columns (int64) drive nut_join_i64 — INNER builds the smaller table; LEFT /
 * RIGHT OUTER, SEMI and ANTI preserve their side — and the columns the plan names are
 * gathered through the join index; the rest of the plan runs on the joined rows.  Outer
 * joins: NULL-extended rows add nothing to an aggregate whose argument reads the other
 * table (its aggregate mask), and the other table's columns may not appear in WHERE,
 * GROUP BY or a scan; SEMI / ANTI expose only the preserved table. */
nut_status nut_plan_execute2(nut_ctx *ctx, const nut_plan *plan, const nut_column *left, int nleft, uint64_t lrows,
                             const nut_column *right, int nright, uint64_t rrows, uint64_t group_hint,
                             nut_result **out);
/* Several JOINs (FROM t0 JOIN t1 ON .. LEFT JOIN t2 ON ..; INNER, LEFT / RIGHT / FULL OUTER,
 * LEFT SEMI / ANTI steps): tables[k] / ncols[k] / nrows[k] = table k in FROM / JOIN order.
 * Each ON compares a column of its table with a column of an earlier one; single-table
 * WHERE conjuncts are pushed down.  A NULL-extended table (LEFT-joined; every earlier one
 * after a RIGHT step; both sides of FULL) is NULL on the rows without a match (a later ON
 * reading it matches nothing there); its columns may only appear inside aggregates, which
 * skip those rows, and in scan projections (NULL there, nut_result_validity).  A SEMI /
 * ANTI step's table only filters (its columns are not output).
 * Plans with at most one JOIN are forwarded to nut_plan_execute / nut_plan_execute2. */
nut_status nut_plan_executen(nut_ctx *ctx, const nut_plan *plan, const nut_column *const *tables, const int *ncols,
                             const uint64_t *nrows, int ntables, uint64_t group_hint, nut_result **out);
/* Result = ncols output columns (the SELECT list, in order) x nrows rows. */
nut_status nut_result_shape(const nut_result *res, uint64_t *nrows, int *ncols);
/* type: nut_type of output column j; name: alias or expression text (owned by res) */
nut_status nut_result_column(const nut_result *res, int j, int *type, const char **name);
/* copy output column j to host (int64 or double; cap in elements) */
nut_status nut_result_to_host(const nut_result *res, int j, void *dst, uint64_t cap);
/* FILTER/SORT results stay in HBM: device pointer of the nrows output values.
 * NUT_ERR_UNSUPPORTED for GROUPBY results (those are materialised on the host). */
nut_status nut_result_device(const nut_result *res, const void **dev);
/* column j of a FILTER / SORT result in HBM (expression-mode scans may project several) */
nut_status nut_result_device_column(const nut_result *r, int j, const void **dev);
/* SQL NULLs of output column j: *dev = nrows 1-byte flags in HBM (1: a value, 0: NULL —
 * a LEFT-joined table's column on a row without a match, or a CASE branch without ELSE),
 * or NULL when the column holds no NULLs (GROUPBY results never do).  A NULL row's value
 * word is 0 (strings: empty). */
nut_status nut_result_validity(const nut_result *r, int j, const uint8_t **dev);
/* the same flags copied to host (all 1 for a column without NULLs; cap in rows) */
nut_status nut_result_validity_to_host(const nut_result *r, int j, uint8_t *dst, uint64_t cap);
/* row of a NUT_T_STR output column (a string group key of a typed table); the bytes
 * are owned by res and not NUL-terminated */
nut_status nut_result_string(const nut_result *res, int j, uint64_t row, const char **s, size_t *len);
void nut_result_free(nut_result *res);

/* ========================================================================
 * Typed tables from CREATE TABLE
 * A CREATE TABLE statement (TableDef, src/parser/ast/stmt.rs; column types
 * ScalarDataType / CompoundDataType, ast/item.rs:14-68) gives an empty table whose
 * columns live in HBM in the executed representation:
 *   Int8..Int64, UInt8..UInt64, Serial*  -> int64   (UInt64 >= 2^63 rejected)
 *   Boolean -> int64 0/1; Date / Datetime -> int64 days / seconds since 1970-01-01
 *   Float32 / Float64 -> f64
 *   String, Chars(n), Dictionary(String) -> int64 codes of the table's dictionary
 *   Enum('a' = 1, ...) -> int64 declared ids;  Nullable(T) -> T (NULLs rejected)
 * Int128/UInt128, Decimal, Uuid, Array, Tuple, Map: NUT_ERR_UNSUPPORTED at create.
 * Plans execute against a table by column name; string constants bind to dictionary
 * codes (= / != / IN, CASE x WHEN 'a'), string group keys come back as NUT_T_STR.
 * ======================================================================== */
typedef struct nut_table nut_table;
typedef enum {
  NUT_COL_INT = 0, NUT_COL_UINT = 1, NUT_COL_FLOAT = 2, NUT_COL_BOOL = 3,
  NUT_COL_DATE = 4, NUT_COL_DATETIME = 5, NUT_COL_STRING = 6, NUT_COL_ENUM = 7
} nut_col_kind;

nut_status nut_table_create(const char *sql, size_t len, nut_table **out);
nut_status nut_table_shape(const nut_table *t, int *ncols, uint64_t *nrows);
/* kind: nut_col_kind; width: bytes per appended host value (numeric kinds) */
nut_status nut_table_column_info(const nut_table *t, int j, const char **name, int *kind, int *width,
                                 int *exec_type);
/* Append n values to column j (host memory -> HBM on ctx's device; narrow integers and
 * Float32 are widened by a GPU kernel).  Numeric kinds: `data` holds n values of the
 * column's width (little-endian; BOOL 1 B; DATE / DATETIME int64).  STRING / ENUM:
 * n UTF-8 strings, string i = data[offsets[i] .. offsets[i+1]).  A table's rows are the
 * rows every column has. */
nut_status nut_table_append(nut_ctx *ctx, nut_table *t, int j, const void *data, const int64_t *offsets,
                            uint64_t n);
/* Execute a plan against the table (binds every plan column by name). */
nut_status nut_table_execute(nut_ctx *ctx, nut_table *t, const nut_plan *plan, uint64_t group_hint,
                             nut_result **out);
/* A JOIN plan over two typed tables (left = FROM, right = JOIN source; nut_plan_execute2
 * semantics).  String columns travel through the join as codes of their own table's
 * dictionary and decode on output; JOIN keys must be integer columns. */
nut_status nut_table_execute2(nut_ctx *ctx, nut_table *left, nut_table *right, const nut_plan *plan,
                              uint64_t group_hint, nut_result **out);
/* A chain of INNER joins over typed tables (tables[0] = FROM, tables[k] = the k-th JOIN
 * source; nut_plan_executen semantics).  Strings as in nut_table_execute2: filters
 * (= / != / IN / LIKE), GROUP BY keys and projections use each column's own dictionary;
 * JOIN keys must be integer columns. */
nut_status nut_table_executen(nut_ctx *ctx, nut_table *const *tables, int ntables, const nut_plan *plan,
                              uint64_t group_hint, nut_result **out);
void nut_table_free(nut_table *t);

#ifdef __cplusplus
}
#endif
#endif /* NUTEXEC_H */
