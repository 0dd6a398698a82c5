/*
 * oracle.h — CPU restatement of the nutexec hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so.  It is the checker, never the thing measured or shipped: the
 * product path (nutdb_amd/, libnutexec.so) never links or calls it.
 *
 * Parity anchor.  The reference (nutdb v0.1.0, /root/reference) is a SQL front end
 * only: there is NO scan / filter / group-by / sort implementation in it
 * (SURVEY.md §0, §2 "ABSENT → build from scratch").  The semantics below are
 * therefore defined by this build and pinned against independent
 * third-party oracles run in the build container — numpy 2.2 (boolean-mask
 * filter, np.sort), pyarrow 25 (Table.group_by().aggregate) and math.fsum
 * (correctly-rounded f64 sums) — whose outputs are committed as fixtures under
 * tests/golden/ by tests/golden/make_golden.py.  With respect to the reference
 * itself, executor parity is "unpinned by construction" (SURVEY.md §8(c)).
 *
 * The literal inputs the reference does hand to the path (the WHERE constant of
 * TPC-H Q1, AST shapes) are pinned by the front-end tests against the reference's
 * own fixtures (tests/golden/sql/N.sql = /root/reference/tests/sql/N.sql).
 */
#ifndef NUT_ORACLE_H
#define NUT_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---- counter-based synthetic data (SURVEY.md §8(d) "splitmix64(seed ⊕ row)") ---- */
uint64_t orc_mix64(uint64_t z);
uint64_t orc_gen_u64(uint64_t seed, uint64_t row);

/* column kinds, identical to include/nutexec.h nut_gen_kind */
enum {
  ORC_GEN_U62 = 0,       /* (int64) (u >> 2)                       uniform [0, 2^62)      */
  ORC_GEN_FULL_I64 = 1,  /* (int64) u                              full-range i64        */
  ORC_GEN_POOL_KEY = 2,  /* pool[u % a], pool[g] = (int64) mix64(g ^ POOL_SALT)         */
  ORC_GEN_DYADIC = 3,    /* (double)(u >> 44) / 64.0               exact-sum f64         */
  ORC_GEN_UNIT_F64 = 4,  /* (double)(u >> 11) * 2^-53              uniform [0,1) f64     */
  ORC_GEN_RANGE_I64 = 5, /* a + (int64)(u % b)                     uniform [a, a+b)      */
  ORC_GEN_RANGE_F64 = 6, /* (double)(a + (int64)(u % b)) / c       decimal-like f64      */
  ORC_GEN_SKEW_KEY = 7,  /* pool[(u % a) >> ((mix64(u) >> 59) * 3 >> 2)]: log-uniform    */
};
/* the pool index of a skewed key (ORC_GEN_SKEW_KEY): index i takes ~1/i of the rows */
#define ORC_SKEW_INDEX(u, a) (((u) % (uint64_t)(a)) >> (((orc_mix64(u) >> 59) * 3) >> 2))
#define ORC_POOL_SALT 0x5DEECE66D2545F49ull
void orc_gen_column(int kind, uint64_t seed, int64_t a, int64_t b, double c,
                    uint64_t row0, uint64_t n, void *out);

/* ---- filter: SELECT col FROM t WHERE col <op> k (row order preserved) ---- */
enum { ORC_LT = 0, ORC_LE = 1, ORC_GT = 2, ORC_GE = 3, ORC_EQ = 4, ORC_NE = 5 };
uint64_t orc_filter_i64(const int64_t *col, uint64_t n, int op, int64_t k, int64_t *out);

/* ---- fused filter -> hash group-by -> aggregate (configs 3, 4) ----
 * Mirrors include/nutexec.h nut_agg_spec field-for-field (plain ints + pointers). */
enum { ORC_T_I64 = 0, ORC_T_F64 = 1 };
enum { ORC_AGG_SUM = 0, ORC_AGG_COUNT = 1, ORC_AGG_MIN = 2, ORC_AGG_MAX = 3 };
enum { ORC_EX_COL = 0, ORC_EX_MUL = 1, ORC_EX_ADD = 2, ORC_EX_SUB = 3,
       ORC_EX_MUL_1M = 4,    /* a * (1 - b)           */
       ORC_EX_MUL_1M_1P = 5  /* a * (1 - b) * (1 + c) */ };

typedef struct {
  uint64_t n;
  int nkeys;                 /* 1 or 2 int64 key columns */
  const int64_t *keys[2];
  int npred;                 /* conjunction of npred terms */
  const void *pred_col[6];
  int pred_type[6];          /* ORC_T_* */
  int pred_op[6];            /* ORC_LT.. */
  int64_t pred_i64[6];
  double pred_f64[6];
  int nvals;                 /* value columns referenced by expressions */
  const void *val_col[8];
  int val_type[8];
  int naggs;
  int agg_op[8];             /* ORC_AGG_* */
  int agg_expr[8];           /* ORC_EX_* */
  int agg_arg[8][3];         /* value-column indices */
  /* expression mode (oracle/expr.py evaluates the programs with numpy): rows pass only
   * where row_mask[i] != 0; aggregate a takes only rows where agg_mask[a][i] != 0.
   * NULL = every row. */
  const uint8_t *row_mask;
  const uint8_t *agg_mask[8];
} orc_agg_spec;

/* Result: groups sorted ascending by key tuple.  Each aggregate is one 64-bit
 * word: f64 bits for SUM/MIN/MAX over f64, int64 for COUNT and i64 SUM/MIN/MAX
 * (i64 SUM wraps two's complement).  out_keys[g*nkeys + j], out_aggs[g*naggs + a].
 * Returns number of groups, or UINT64_MAX if cap is too small.
 * f64 sums are Neumaier-compensated (≈ correctly rounded). nthreads<=0: all cores. */
uint64_t orc_groupby(const orc_agg_spec *spec, uint64_t cap, int64_t *out_keys,
                     uint64_t *out_aggs, int nthreads);
/* The same result by one fixed method: per-thread tables over the row chunks, merged into
 * thread 0's in thread order.  orc_groupby runs this for few groups; for many (a sample
 * estimate >= 16384, >= 2^22 rows) it range-partitions the rows and merges per partition
 * on every thread with the same per-group order — bitwise the same result
 * (tests/test_oracle_golden.py checks the two against each other). */
uint64_t orc_groupby_tables(const orc_agg_spec *spec, uint64_t cap, int64_t *out_keys,
                            uint64_t *out_aggs, int nthreads);

/* ---- indexed group-by of the synthetic pool-key workload (config 3 at full size) ----
 * SELECT key, SUM(val), COUNT(*), MIN(val), MAX(val) GROUP BY key over rows
 * [row0, row0+n) of key = ORC_GEN_POOL_KEY(key_seed, a = groups), val =
 * ORC_GEN_DYADIC(val_seed): accumulated by pool index in dense arrays (exact, no hash
 * table), so 1e9 rows x 1e7 groups take seconds.  out_keys[m], out_words[m][4] (f64 bits
 * of SUM, COUNT, f64 bits of MIN, MAX), groups ordered by key; returns m (groups with at
 * least one row), UINT64_MAX on allocation failure.  Pinned against orc_groupby on the
 * same generated columns (tests/test_oracle_golden.py). */
uint64_t orc_groupby_pool_dyadic(uint64_t key_seed, uint64_t groups, uint64_t val_seed, uint64_t row0, uint64_t n,
                                 int64_t *out_keys, uint64_t *out_words, int nthreads);
/* the same for kind ORC_GEN_POOL_KEY or ORC_GEN_SKEW_KEY keys (the skewed workload's
 * full-size checker) */
uint64_t orc_groupby_pool_dyadic_kind(int kind, uint64_t key_seed, uint64_t groups, uint64_t val_seed, uint64_t row0,
                                      uint64_t n, int64_t *out_keys, uint64_t *out_words, int nthreads);

/* ---- sort: ascending int64 ---- */
void orc_sort_i64(const int64_t *in, int64_t *out, uint64_t n, int nthreads);
/* Hash equi-join, nut_join_i64 semantics (type 0 INNER, 1 LEFT, 2 SEMI, 3 ANTI): pairs in
 * probe-row order, build rows of one probe row in unspecified order, -1 = no build row.
 * Writes at most cap pairs and returns the pair count. */
uint64_t orc_join_i64(const int64_t *build, uint64_t nb, const int64_t *probe, uint64_t np, int type,
                      int64_t *out_p, int64_t *out_b, uint64_t cap);

/* ---- expression programs, integer subset, on every host core (bench CPU baseline) ----
 * RPN nodes (op, arg, v) with oracle/expr.py's op numbering: col (int64 columns), i64,
 * add / sub / mul (wrapping), lt le gt ge eq ne, and / or / xor / not (non-zero = true),
 * bitand / bitor / bitxor / bitnot, if.  None of these can fail a row, so the values are
 * those of expr.py's eval_prog (bools as 0/1).  Row blocks of 2048 on OpenMP threads.
 * Returns 0, or -1 for a program outside the subset (nothing written). */
int orc_eval_int(const int32_t *op, const int32_t *arg, const int64_t *v, int nnodes, const int64_t *const *cols,
                 int ncols, uint64_t n, int64_t *out);

/* order-independent multiset hash (sum of mix64 of each element), for sort parity */
uint64_t orc_multiset_hash_i64(const int64_t *v, uint64_t n);

int orc_max_threads(void);

#ifdef __cplusplus
}
#endif
#endif
