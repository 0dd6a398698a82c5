// agg_ops.hpp — argument block, compiled query shapes and per-row operators of the
// streaming filter -> group-by -> aggregate kernel (agg_kernel.hpp).
//
// One pass over the columns:
//   * each lane holds FOUR rows per iteration (two 16-B loads per column); every
//     uniform decision (predicate op, aggregate kind, expression) is taken once per
//     four rows, and for the compiled query shapes (Fixed<>) at compile time — the
//     generic kernel was measured SALU/VALU-bound on exactly these switches;
//   * per-workgroup hash table in LDS (slot words + one 64-bit word per aggregate,
//     structure of arrays).  Keys are found lock-free; NEW keys of tables that publish
//     more than the slot word (two-key tuples, private ids) are inserted under a
//     block-level LDS lock, so nothing is ever half-published and no entry is wasted;
//   * PRIV (tiny group counts): the first P groups of a block get per-thread private
//     accumulators in LDS laid out [group][agg][thread] — plain read-add-write, no
//     atomics, no bank conflicts — reduced once per block.  Measured motivation: Q1's
//     6 groups put 64 lanes on 6 addresses (11 extra LDS cycles per LDS instruction);
//   * keys the block table does not admit go to the global table (g_row, rare);
//   * at block end the table is merged into the global (HBM) table.
#pragma once

#include "gtable.hpp"

namespace nut {

constexpr int kPrivMax = 8;  // private groups per thread (upper bound)
constexpr int kMaxCols = NUT_MAX_PROG_COLS;  // value columns a kernel can load
constexpr int kMaxConst = 64;                // expression constants (kernel arguments)

struct AggArgs {
  uint64_t n;
  const uint64_t *keys[2];
  const uint64_t *pred_col[NUT_MAX_PRED];
  uint64_t pred_k[NUT_MAX_PRED];  // constant bits
  int32_t pred_type[NUT_MAX_PRED];
  int32_t pred_op[NUT_MAX_PRED];
  const uint64_t *val_col[kMaxCols];  // expression shapes load every program column here
  int32_t npred, nvals, naggs;
  uint32_t kinds;                 // 4 bits per aggregate kind
  int32_t expr[NUT_MAX_AGGS];
  int32_t arg[NUT_MAX_AGGS][3];
  uint32_t lds_cap;               // power of two, 0 = no LDS table
  uint32_t lds_limit;             // claims admitted before the table closes
  int32_t lds_log2;
  int32_t priv;                   // private groups per thread (PRIV kernels)
  int32_t vec;                    // all columns 16-B aligned: vector loads
  int32_t nokey;                  // global aggregate: no key column, every key is 0
  int32_t pred_nset[NUT_MAX_PRED];                 // NUT_IN / NUT_NOT_IN set sizes
  uint64_t pred_set[NUT_MAX_PRED][NUT_MAX_SET];    // set values (bits)
  uint64_t kc[kMaxConst];         // expression constants (bits), read by generated shapes
  const GTable *gt;               // device copy of the global table descriptor
  // Partitioned aggregation (gpart.hip), for more groups than the on-chip tables hold.
  // Spill mode (sp_counts != 0, lds_cap = 0): every row passing WHERE is appended to the
  // staged arrays sp_cols = {-, k1, k2, value arrays...} instead of the global table,
  // block b at [b * sp_region, ...) (an LDS cursor; the count lands in sp_counts[b]);
  // aggregate a's value goes to array 3 + sp_map[a] (-1: not staged).
  uint64_t *sp_cols[3 + NUT_MAX_VALS];  // [0] unused (the partition hash is recomputed)
  unsigned long long *sp_counts;
  unsigned long long *sp_hist;   // [256] histogram of the key hash's top byte (level 0)
  uint64_t sp_region;
  int32_t sp_map[NUT_MAX_AGGS];
  // Segment mode (seg_off != 0): block b folds rows [seg_off[2b], seg_off[2b+1]) only.
  const uint64_t *seg_off;
  const uint64_t *seg_end;  // non-null: block b's rows are [seg_off[b], seg_end[b]) instead
  const uint64_t *seg_cut;  // non-null (with seg_end): ... [seg_off[b], min(seg_end[b], seg_cut[b]))
  // dense (segment mode, one key, every segment a whole partition): a block's groups are
  // final, so they are appended to the table's first slots instead of hashed into it
  int32_t dense, pad_;
  // dense staging (the ordered group-by): block b's groups (the empty-marker key's included)
  // go to table slots [(dbase + b) * dregion, + count) in any order, count to dcount[b]
  unsigned long long *dcount;
  uint64_t dregion, dbase;
};

// ------------------------------------------------------------------ query shapes
// A shape answers what the kernel would otherwise read from AggArgs at run time.
//
// kProg shapes (generated per query and compiled at run time, jit.cpp) also provide
//   where(p, v, r, err)     -> bool       the WHERE program of row r
//   value(p, a, v, r, err)  -> u64 bits   aggregate a's argument
//   valid(p, a, v, r, err)  -> bool       aggregate a's row mask
// over v = the loaded columns; err is set by a failing integer division.
struct NoProg {
  static constexpr bool kProg = false;
  template <class V>
  __device__ static bool where(const AggArgs &, const V &, int, bool &) { return true; }
  template <class V>
  __device__ static uint64_t value(const AggArgs &, int, const V &, int, bool &) { return 0; }
  template <class V>
  __device__ static bool valid(const AggArgs &, int, const V &, int, bool &) { return true; }
};

struct Generic : NoProg {
  static constexpr int MP = NUT_MAX_PRED, MV = NUT_MAX_VALS, MA = NUT_MAX_AGGS;
  __device__ static int np(const AggArgs &p) { return p.npred; }
  __device__ static int nv(const AggArgs &p) { return p.nvals; }
  __device__ static int na(const AggArgs &p) { return p.naggs; }
  __device__ static int kind(const AggArgs &p, int a) { return kind_at(p.kinds, a); }
  __device__ static int expr(const AggArgs &p, int a) { return p.expr[a]; }
  __device__ static int arg(const AggArgs &p, int a, int j) { return p.arg[a][j]; }
  __device__ static int ptype(const AggArgs &p, int t) { return p.pred_type[t]; }
  __device__ static int pop(const AggArgs &p, int t) { return p.pred_op[t]; }
};

// packed: KINDS/EXPRS 4 bits per aggregate, ARGS 6 bits (3 x 2) per aggregate,
// PREDS 4 bits per predicate term (type << 3 | op)
template <int NP, int NV, int NA, uint32_t KINDS, uint32_t EXPRS, uint64_t ARGS, uint32_t PREDS>
struct Fixed : NoProg {
  static constexpr int MP = NP, MV = NV, MA = NA;
  static constexpr uint32_t kKinds = KINDS, kExprs = EXPRS, kPreds = PREDS;
  static constexpr uint64_t kArgs = ARGS;
  __device__ static constexpr int np(const AggArgs &) { return NP; }
  __device__ static constexpr int nv(const AggArgs &) { return NV; }
  __device__ static constexpr int na(const AggArgs &) { return NA; }
  __device__ static constexpr int kind(const AggArgs &, int a) { return (int)((KINDS >> (4 * a)) & 15u); }
  __device__ static constexpr int expr(const AggArgs &, int a) { return (int)((EXPRS >> (4 * a)) & 15u); }
  __device__ static constexpr int arg(const AggArgs &, int a, int j) { return (int)((ARGS >> (6 * a + 2 * j)) & 3u); }
  __device__ static constexpr int ptype(const AggArgs &, int t) { return (int)((PREDS >> (4 * t + 3)) & 1u); }
  __device__ static constexpr int pop(const AggArgs &, int t) { return (int)((PREDS >> (4 * t)) & 7u); }
};

#define NUT_K4(a, b, c, d) ((uint32_t)(a) | ((uint32_t)(b) << 4) | ((uint32_t)(c) << 8) | ((uint32_t)(d) << 12))
#define NUT_A3(x, y, z) ((uint64_t)(x) | ((uint64_t)(y) << 2) | ((uint64_t)(z) << 4))
// TPC-H Q1 shape: WHERE i64 <= k; SUM(v0), SUM(v1), SUM(v1*(1-v2)), COUNT(*)
using ShapeQ1 = Fixed<1, 3, 4, NUT_K4(AK_SUM_F64, AK_SUM_F64, AK_SUM_F64, AK_COUNT),
                      NUT_K4(NUT_EX_COL, NUT_EX_COL, NUT_EX_MUL_1M, NUT_EX_COL),
                      NUT_A3(0, 0, 0) | (NUT_A3(1, 0, 0) << 6) | (NUT_A3(1, 2, 0) << 12),
                      (NUT_T_I64 << 3) | NUT_LE>;
// config 3: SUM(v0)
using ShapeSum = Fixed<0, 1, 1, AK_SUM_F64, NUT_EX_COL, 0, 0>;
// config 3 variants: SUM, COUNT / SUM, COUNT, MIN, MAX over v0
using ShapeSumCount = Fixed<0, 1, 2, NUT_K4(AK_SUM_F64, AK_COUNT, 0, 0), 0, 0, 0>;
using ShapeAll4 = Fixed<0, 1, 4, NUT_K4(AK_SUM_F64, AK_COUNT, AK_MIN_F64, AK_MAX_F64), 0, 0, 0>;

// ------------------------------------------------------------------ per-kind ops
template <int V>
struct IC {
  static constexpr int value = V;
};

// call f(IC<kind>{}) with the aggregate kind as a compile-time constant
template <class F>
__device__ __forceinline__ void with_kind(int k, F &&f) {
  switch (k) {
    case AK_SUM_F64: f(IC<AK_SUM_F64>{}); break;
    case AK_SUM_I64: f(IC<AK_SUM_I64>{}); break;
    case AK_COUNT: f(IC<AK_COUNT>{}); break;
    case AK_MIN_F64: f(IC<AK_MIN_F64>{}); break;
    case AK_MAX_F64: f(IC<AK_MAX_F64>{}); break;
    case AK_MIN_I64: f(IC<AK_MIN_I64>{}); break;
    default: f(IC<AK_MAX_I64>{}); break;
  }
}

// fold one row value x into an accumulator word (plain, non-atomic)
template <int K>
__device__ __forceinline__ uint64_t fold(uint64_t acc, uint64_t x) {
  if constexpr (K == AK_SUM_F64) return as_u64(as_f64(acc) + as_f64(x));
  else if constexpr (K == AK_SUM_I64) return acc + x;
  else if constexpr (K == AK_COUNT) return acc + 1;
  else if constexpr (K == AK_MIN_F64) { uint64_t o = f64_to_ord(x); return o < acc ? o : acc; }
  else if constexpr (K == AK_MAX_F64) { uint64_t o = f64_to_ord(x); return o > acc ? o : acc; }
  else if constexpr (K == AK_MIN_I64) return (int64_t)x < (int64_t)acc ? x : acc;
  else return (int64_t)x > (int64_t)acc ? x : acc;
}
// combine two accumulator words of the same kind (plain)
template <int K>
__device__ __forceinline__ uint64_t combine(uint64_t a, uint64_t b) {
  if constexpr (K == AK_SUM_F64) return as_u64(as_f64(a) + as_f64(b));
  else if constexpr (K == AK_SUM_I64 || K == AK_COUNT) return a + b;
  else if constexpr (K == AK_MIN_F64) return a < b ? a : b;
  else if constexpr (K == AK_MAX_F64) return a > b ? a : b;
  else if constexpr (K == AK_MIN_I64) return (int64_t)a < (int64_t)b ? a : b;
  else return (int64_t)a > (int64_t)b ? a : b;
}
// atomic fold of one row value into a shared (LDS or global) word
template <int K>
__device__ __forceinline__ void fold_atomic(uint64_t *w, uint64_t x) {
  if constexpr (K == AK_SUM_F64) unsafeAtomicAdd((double *)w, as_f64(x));
  else if constexpr (K == AK_SUM_I64) atomicAdd((unsigned long long *)w, (unsigned long long)x);
  else if constexpr (K == AK_COUNT) atomicAdd((unsigned long long *)w, 1ull);
  else if constexpr (K == AK_MIN_F64) atomicMin((unsigned long long *)w, (unsigned long long)f64_to_ord(x));
  else if constexpr (K == AK_MAX_F64) atomicMax((unsigned long long *)w, (unsigned long long)f64_to_ord(x));
  else if constexpr (K == AK_MIN_I64) atomicMin((long long *)w, (long long)x);
  else atomicMax((long long *)w, (long long)x);
}

template <int OP, int TY>
__device__ __forceinline__ bool pred1(uint64_t v, uint64_t k) {
  if constexpr (TY == NUT_T_I64) {
    const int64_t a = (int64_t)v, b = (int64_t)k;
    if constexpr (OP == NUT_LT) return a < b;
    else if constexpr (OP == NUT_LE) return a <= b;
    else if constexpr (OP == NUT_GT) return a > b;
    else if constexpr (OP == NUT_GE) return a >= b;
    else if constexpr (OP == NUT_EQ) return a == b;
    else return a != b;
  } else {
    const double a = as_f64(v), b = as_f64(k);
    if constexpr (OP == NUT_LT) return a < b;
    else if constexpr (OP == NUT_LE) return a <= b;
    else if constexpr (OP == NUT_GT) return a > b;
    else if constexpr (OP == NUT_GE) return a >= b;
    else if constexpr (OP == NUT_EQ) return a == b;
    else return a != b;
  }
}

// call f(IC<op>{}, IC<type>{}) with a predicate term's operator and column type
template <class F>
__device__ __forceinline__ void with_pred(int ty, int op, F &&f) {
  if (ty == NUT_T_I64) {
    switch (op) {
      case NUT_LT: f(IC<NUT_LT>{}, IC<NUT_T_I64>{}); break;
      case NUT_LE: f(IC<NUT_LE>{}, IC<NUT_T_I64>{}); break;
      case NUT_GT: f(IC<NUT_GT>{}, IC<NUT_T_I64>{}); break;
      case NUT_GE: f(IC<NUT_GE>{}, IC<NUT_T_I64>{}); break;
      case NUT_EQ: f(IC<NUT_EQ>{}, IC<NUT_T_I64>{}); break;
      default: f(IC<NUT_NE>{}, IC<NUT_T_I64>{}); break;
    }
  } else {
    switch (op) {
      case NUT_LT: f(IC<NUT_LT>{}, IC<NUT_T_F64>{}); break;
      case NUT_LE: f(IC<NUT_LE>{}, IC<NUT_T_F64>{}); break;
      case NUT_GT: f(IC<NUT_GT>{}, IC<NUT_T_F64>{}); break;
      case NUT_GE: f(IC<NUT_GE>{}, IC<NUT_T_F64>{}); break;
      case NUT_EQ: f(IC<NUT_EQ>{}, IC<NUT_T_F64>{}); break;
      default: f(IC<NUT_NE>{}, IC<NUT_T_F64>{}); break;
    }
  }
}

template <int E>
__device__ __forceinline__ uint64_t eval(uint64_t x, uint64_t y, uint64_t z) {
  if constexpr (E == NUT_EX_COL) return x;
  else {
    const double a = as_f64(x), b = as_f64(y);
    double r;
    if constexpr (E == NUT_EX_MUL) r = __dmul_rn(a, b);
    else if constexpr (E == NUT_EX_ADD) r = __dadd_rn(a, b);
    else if constexpr (E == NUT_EX_SUB) r = __dsub_rn(a, b);
    else if constexpr (E == NUT_EX_MUL_1M) r = __dmul_rn(a, __dsub_rn(1.0, b));
    else r = __dmul_rn(__dmul_rn(a, __dsub_rn(1.0, b)), __dadd_rn(1.0, as_f64(z)));
    return as_u64(r);
  }
}

// call f(IC<expr>{}) with an aggregate's expression as a compile-time constant
template <class F>
__device__ __forceinline__ void with_expr(int e, F &&f) {
  switch (e) {
    case NUT_EX_COL: f(IC<NUT_EX_COL>{}); break;
    case NUT_EX_MUL: f(IC<NUT_EX_MUL>{}); break;
    case NUT_EX_ADD: f(IC<NUT_EX_ADD>{}); break;
    case NUT_EX_SUB: f(IC<NUT_EX_SUB>{}); break;
    case NUT_EX_MUL_1M: f(IC<NUT_EX_MUL_1M>{}); break;
    default: f(IC<NUT_EX_MUL_1M_1P>{}); break;
  }
}

// ------------------------------------------------------------------ global fall-back
// rows whose key the block table did not admit (rare; out of line keeps the loop small)
template <int NK>
__device__ __noinline__ void g_row(const GTable *__restrict__ gtp, int64_t k1, int64_t k2, uint32_t amask,
                                   uint64_t a0, uint64_t a1, uint64_t a2, uint64_t a3, uint64_t a4, uint64_t a5,
                                   uint64_t a6, uint64_t a7) {
  const GTable t = *gtp;
  int64_t gs = g_find<NK>(t, key_hash<NK>(k1, k2), k1, k2);
  if (gs < 0) return;
  const uint64_t stride = t.cap + 1;
  const uint64_t av[8] = {a0, a1, a2, a3, a4, a5, a6, a7};
#pragma unroll
  for (int a = 0; a < NUT_MAX_AGGS; ++a)
    if (a < t.naggs && ((amask >> a) & 1u)) agg_update(&t.agg[a * stride + gs], kind_at(t.kinds, a), av[a]);
}


}  // namespace nut
