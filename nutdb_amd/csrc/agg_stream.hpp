// agg_stream.hpp — the streaming filter -> group-by -> aggregate kernel.
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

struct AggArgs {
  uint64_t n;
  const uint64_t *keys[2];
  const uint64_t *pred_col[NUT_MAX_PRED];
  uint64_t pred_k[NUT_MAX_PRED];  // constant bits
  int32_t pred_type[NUT_MAX_PRED];
  int32_t pred_op[NUT_MAX_PRED];
  const uint64_t *val_col[NUT_MAX_VALS];
  int32_t npred, nvals, naggs;
  uint32_t kinds;                 // 4 bits per aggregate kind
  int32_t expr[NUT_MAX_AGGS];
  int32_t arg[NUT_MAX_AGGS][3];
  uint32_t lds_cap;               // power of two, 0 = no LDS table
  uint32_t lds_limit;             // claims admitted before the table closes
  int32_t lds_log2;
  int32_t priv;                   // private groups per thread (PRIV kernels)
  int32_t vec;                    // all columns 16-B aligned: vector loads
  const GTable *gt;               // device copy of the global table descriptor
};

// ------------------------------------------------------------------ query shapes
// A shape answers what the kernel would otherwise read from AggArgs at run time.
struct Generic {
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
struct Fixed {
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
__device__ __noinline__ void g_row(const GTable *__restrict__ gtp, int64_t k1, int64_t k2, uint64_t a0,
                                   uint64_t a1, uint64_t a2, uint64_t a3, uint64_t a4, uint64_t a5, uint64_t a6,
                                   uint64_t a7) {
  const GTable t = *gtp;
  int64_t gs = g_find<NK>(t, key_hash<NK>(k1, k2), k1, k2);
  if (gs < 0) return;
  const uint64_t stride = t.cap + 1;
  const uint64_t av[8] = {a0, a1, a2, a3, a4, a5, a6, a7};
#pragma unroll
  for (int a = 0; a < NUT_MAX_AGGS; ++a)
    if (a < t.naggs) agg_update(&t.agg[a * stride + gs], kind_at(t.kinds, a), av[a]);
}

// ------------------------------------------------------------------ LDS table
// Layout (dynamic LDS, this order, 16-B aligned):
//   slot[cap+1] u64 | agg[na][cap+1] u64 | k1,k2[cap+1] i64 (NK=2) | did[cap+1] u32 (PRIV)
//   | dslot[kPrivMax] u32 (PRIV) | ctl[4] u32 | pad16 | priv[P][na][BD] u64 (PRIV)
enum { CTL_CLAIMED = 0, CTL_SPECIAL = 1, CTL_LOCK = 2, CTL_NDENSE = 3 };
constexpr uint32_t kNoDense = 0xFFFFFFFFu;

struct LTable {
  uint64_t *slot, *agg;
  int64_t *k1, *k2;
  uint32_t *did, *dslot, *ctl;
  uint64_t *priv;
};

__host__ __device__ inline size_t lds_layout(uint32_t cap, int nk, int na, bool privm, int P, int bd,
                                             size_t *o_k1, size_t *o_did, size_t *o_dslot, size_t *o_ctl,
                                             size_t *o_priv) {
  const size_t stride = cap + 1;
  size_t o = stride * 8 * (1 + (size_t)na);
  *o_k1 = o;
  if (nk == 2) o += stride * 16;
  *o_did = o;
  if (privm) o += stride * 4;
  *o_dslot = o;
  if (privm) o += kPrivMax * 4;
  *o_ctl = o;
  o += 16;
  o = (o + 15) & ~size_t(15);
  *o_priv = o;
  if (privm) o += (size_t)P * na * bd * 8;
  return (o + 15) & ~size_t(15);
}

// multiply-shift home slot; two-key hash nudged off the empty marker
template <int NK>
__device__ __forceinline__ uint64_t lkey(int64_t k1, int64_t k2) {
  if (NK == 1) return (uint64_t)k1;
  uint64_t h = (uint64_t)k1 * kGolden ^ (((uint64_t)k2 + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full);
  h ^= h >> 29;
  return h == kEmpty ? h ^ 1ull : h;
}

// Lock-free lookup along the probe chain: slot index, or -1 (reached an empty slot at
// *empty_at) or -2 (chain exhausted).
template <int NK, bool ACQ>
__device__ __forceinline__ int32_t l_walk(const LTable &t, uint32_t cap, int log2cap, uint64_t w, int64_t k1,
                                          int64_t k2, uint32_t &empty_at) {
  uint32_t s = slot_of(w, log2cap);
  for (uint32_t probe = 0; probe < cap; ++probe) {
    uint64_t cur = ACQ ? __hip_atomic_load(&t.slot[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) : t.slot[s];
    if (cur == w && (NK == 1 || (t.k1[s] == k1 && t.k2[s] == k2))) return (int32_t)s;
    if (cur == kEmpty) {
      empty_at = s;
      return -1;
    }
    s = (s + 1) & (cap - 1);
  }
  return -2;
}

// Find or insert: returns the slot (>= 0), or -1 (not admitted: global table).
// LOCKED (two-key or private ids): inserts are serialised by a block lock and publish
// the slot word last; otherwise a CAS on the slot word claims it.
template <int NK, bool LOCKED>
__device__ __forceinline__ int32_t l_find(const LTable &t, const AggArgs &p, uint64_t w, int64_t k1, int64_t k2) {
  const uint32_t cap = p.lds_cap;
  if (NK == 1 && w == kEmpty) {
    t.ctl[CTL_SPECIAL] = 1u;
    return (int32_t)cap;
  }
  uint32_t e = 0;
  int32_t s = l_walk<NK, LOCKED>(t, cap, p.lds_log2, w, k1, k2, e);
  if (s >= 0 || s == -2) return s >= 0 ? s : -1;
  if (!LOCKED) {
    // CAS claim along the chain from the first empty slot
    for (uint32_t probe = 0; probe < cap; ++probe) {
      uint64_t cur = t.slot[e];
      if (cur == w) return (int32_t)e;
      if (cur == kEmpty) {
        if (*(volatile uint32_t *)&t.ctl[CTL_CLAIMED] >= p.lds_limit) return -1;
        cur = atomicCAS((unsigned long long *)&t.slot[e], (unsigned long long)kEmpty, (unsigned long long)w);
        if (cur == kEmpty) {
          atomicAdd(&t.ctl[CTL_CLAIMED], 1u);
          return (int32_t)e;
        }
        if (cur == w) return (int32_t)e;
      }
      e = (e + 1) & (cap - 1);
    }
    return -1;
  }
  // locked insert: every waiting lane of the wave retries until it has run its own
  // critical section; the lock holder's section runs in the same pass (no SIMT
  // deadlock), other waves simply retry
  int32_t res = -1;
  bool done = false;
  for (uint32_t spins = 0;; ++spins) {
    if (!done) {
      if (__hip_atomic_exchange(&t.ctl[CTL_LOCK], 1u, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
        uint32_t e2 = 0;
        res = l_walk<NK, true>(t, cap, p.lds_log2, w, k1, k2, e2);
        if (res == -1) {
          res = -1;
          if (t.ctl[CTL_CLAIMED] < p.lds_limit) {
            if (NK == 2) {
              t.k1[e2] = k1;
              t.k2[e2] = k2;
            }
            if (t.did) {
              uint32_t d = t.ctl[CTL_NDENSE];
              if (d < (uint32_t)p.priv) {
                t.dslot[d] = e2;
                t.ctl[CTL_NDENSE] = d + 1;
              } else {
                d = kNoDense;
              }
              t.did[e2] = d;
            }
            t.ctl[CTL_CLAIMED] += 1u;
            __hip_atomic_store(&t.slot[e2], w, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            res = (int32_t)e2;
          }
        } else if (res == -2) {
          res = -1;
        }
        __hip_atomic_store(&t.ctl[CTL_LOCK], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        done = true;
      }
    }
    if (__all(done) || spins > (1u << 20)) break;
    __builtin_amdgcn_s_sleep(1);
  }
  return done ? res : -1;
}

// ------------------------------------------------------------------ the kernel
__device__ __forceinline__ void load2(const uint64_t *col, uint64_t i, bool vec, uint64_t &x, uint64_t &y) {
  if (vec) {
    u64x2 v = *reinterpret_cast<const u64x2 *>(col + i);
    x = v.x;
    y = v.y;
  } else {
    x = col[i];
    y = col[i + 1];
  }
}
__device__ __forceinline__ void load2_tail(const uint64_t *col, uint64_t i, uint64_t n, uint64_t &x, uint64_t &y) {
  x = i < n ? col[i] : 0;
  y = i + 1 < n ? col[i + 1] : 0;
}

template <class S>
struct Rows {
  static constexpr int R = 4;
  uint64_t k1[R], k2[R];
  uint64_t pv[S::MP > 0 ? S::MP : 1][R];
  uint64_t vv[S::MV > 0 ? S::MV : 1][R];
};

// load rows {i0, i0+1, i1, i1+1}
template <int NK, class S, bool TAIL>
__device__ __forceinline__ void load_rows(const AggArgs &p, uint64_t i0, uint64_t i1, Rows<S> &x) {
  auto ld = [&](const uint64_t *col, uint64_t (&d)[4]) {
    if (TAIL) {
      load2_tail(col, i0, p.n, d[0], d[1]);
      load2_tail(col, i1, p.n, d[2], d[3]);
    } else {
      load2(col, i0, p.vec, d[0], d[1]);
      load2(col, i1, p.vec, d[2], d[3]);
    }
  };
#pragma unroll
  for (int t = 0; t < S::MP; ++t)
    if (t < S::np(p)) ld(p.pred_col[t], x.pv[t]);
  ld(p.keys[0], x.k1);
  if (NK == 2) ld(p.keys[1], x.k2);
#pragma unroll
  for (int c = 0; c < S::MV; ++c)
    if (c < S::nv(p)) ld(p.val_col[c], x.vv[c]);
}

template <int NK, bool PRIV, int BD, class S, bool TAIL>
__device__ __forceinline__ void consume_rows(const AggArgs &p, const LTable &lt, uint64_t i0, uint64_t i1,
                                             const Rows<S> &x) {
  constexpr int R = 4;
  constexpr bool LOCKED = NK == 2 || PRIV;
  bool ok[R];
#pragma unroll
  for (int r = 0; r < R; ++r) ok[r] = !TAIL || ((r < 2 ? i0 : i1) + (r & 1)) < p.n;
  // WHERE: one decision per term per four rows
#pragma unroll
  for (int t = 0; t < S::MP; ++t) {
    if (t < S::np(p)) {
      const uint64_t k = p.pred_k[t];
      with_pred(S::ptype(p, t), S::pop(p, t), [&](auto OPC, auto TYC) {
        constexpr int OP = decltype(OPC)::value, TY = decltype(TYC)::value;
#pragma unroll
        for (int r = 0; r < R; ++r) ok[r] = ok[r] && pred1<OP, TY>(x.pv[t][r], k);
      });
    }
  }
  // aggregate inputs
  uint64_t av[S::MA][R];
#pragma unroll
  for (int a = 0; a < S::MA; ++a) {
#pragma unroll
    for (int r = 0; r < R; ++r) av[a][r] = 0;
    if (a < S::na(p) && S::kind(p, a) != AK_COUNT) {
      const int a0 = S::arg(p, a, 0), a1 = S::arg(p, a, 1), a2 = S::arg(p, a, 2);
      with_expr(S::expr(p, a), [&](auto EC) {
        constexpr int E = decltype(EC)::value;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          auto pick = [&](int c) {
            uint64_t v = x.vv[0][r];
#pragma unroll
            for (int q = 1; q < S::MV; ++q) v = c == q ? x.vv[q][r] : v;
            return v;
          };
          av[a][r] = eval<E>(pick(a0), pick(a1), pick(a2));
        }
      });
    }
  }
  // GROUP BY: find each row's slot
  int32_t sl[R];
  uint32_t dd[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    sl[r] = -2;
    dd[r] = kNoDense;
    if (ok[r]) {
      const uint64_t w = lkey<NK>((int64_t)x.k1[r], (int64_t)x.k2[r]);
      sl[r] = p.lds_cap ? l_find<NK, LOCKED>(lt, p, w, (int64_t)x.k1[r], (int64_t)x.k2[r]) : -1;
      if (PRIV && sl[r] >= 0 && sl[r] < (int32_t)p.lds_cap) dd[r] = lt.did[sl[r]];
    }
  }
  // fold
  const uint32_t stride = p.lds_cap + 1;
#pragma unroll
  for (int a = 0; a < S::MA; ++a) {
    if (a < S::na(p)) {
      with_kind(S::kind(p, a), [&](auto KC) {
        constexpr int K = decltype(KC)::value;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (sl[r] >= 0) {
            if (PRIV && dd[r] != kNoDense) {
              uint64_t *w = &lt.priv[((size_t)dd[r] * S::na(p) + a) * BD + threadIdx.x];
              *w = fold<K>(*w, av[a][r]);
            } else {
              fold_atomic<K>(&lt.agg[a * stride + sl[r]], av[a][r]);
            }
          }
        }
      });
    }
  }
  // rows the block table did not admit
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (sl[r] == -1) {
      uint64_t g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int a = 0; a < S::MA && a < 8; ++a) g[a] = av[a][r];
      g_row<NK>(p.gt, (int64_t)x.k1[r], (int64_t)x.k2[r], g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7]);
    }
  }
}

template <int NK, bool PRIV, int BD, class S>
__global__ __launch_bounds__(BD) void agg_kernel(AggArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const uint32_t cap = p.lds_cap;
  const uint32_t stride = cap + 1;
  const int na = S::na(p);
  LTable lt;
  {
    size_t o_k1, o_did, o_dslot, o_ctl, o_priv;
    lds_layout(cap, NK, na, PRIV, p.priv, BD, &o_k1, &o_did, &o_dslot, &o_ctl, &o_priv);
    char *b = (char *)smem;
    lt.slot = (uint64_t *)b;
    lt.agg = lt.slot + stride;
    lt.k1 = (int64_t *)(b + o_k1);
    lt.k2 = lt.k1 + stride;
    lt.did = PRIV ? (uint32_t *)(b + o_did) : nullptr;
    lt.dslot = (uint32_t *)(b + o_dslot);
    lt.ctl = (uint32_t *)(b + o_ctl);
    lt.priv = (uint64_t *)(b + o_priv);
  }
  if (cap) {
    for (uint32_t s = threadIdx.x; s < stride; s += BD) {
      lt.slot[s] = kEmpty;
#pragma unroll
      for (int a = 0; a < S::MA; ++a)
        if (a < na) lt.agg[a * stride + s] = agg_init(S::kind(p, a));
      if (PRIV) lt.did[s] = kNoDense;
    }
    if (threadIdx.x < 4) lt.ctl[threadIdx.x] = 0;
    if (PRIV) {
#pragma unroll
      for (int a = 0; a < S::MA; ++a)
        if (a < na) {
          const uint64_t init = agg_init(S::kind(p, a));
          for (int d = 0; d < p.priv; ++d) lt.priv[((size_t)d * na + a) * BD + threadIdx.x] = init;
        }
    }
    __syncthreads();
  }

  // grid-stride over row pairs; each lane takes pairs q and q + gstride (4 rows)
  const uint64_t npairs = (p.n + 1) / 2;
  const uint64_t full_pairs = p.n / 2;
  const uint64_t gstride = (uint64_t)gridDim.x * BD;
  uint64_t q = (uint64_t)blockIdx.x * BD + threadIdx.x;
  for (; q + gstride < full_pairs; q += 2 * gstride) {
    Rows<S> x;
    load_rows<NK, S, false>(p, 2 * q, 2 * (q + gstride), x);
    consume_rows<NK, PRIV, BD, S, false>(p, lt, 2 * q, 2 * (q + gstride), x);
  }
  if (q < npairs) {  // last partial step: at most two pairs left for this lane
    const uint64_t q1 = q + gstride < npairs ? q + gstride : q;
    Rows<S> x;
    load_rows<NK, S, true>(p, 2 * q, 2 * q1, x);
    // the duplicate pair (q1 == q) is masked out by pretending it is past the end
    consume_rows<NK, PRIV, BD, S, true>(p, lt, 2 * q, q1 == q ? p.n : 2 * q1, x);
  }

  if (!cap) return;
  __syncthreads();
  if (PRIV) {
    // reduce each (group, aggregate) column of the private accumulators: 8 threads per
    // pair, fixed order, then one LDS atomic merge into the shared slot
    const uint32_t nd = min(lt.ctl[CTL_NDENSE], (uint32_t)p.priv);
    const int part = threadIdx.x & 7;
    for (uint32_t pi = threadIdx.x >> 3; pi < nd * (uint32_t)na; pi += BD / 8) {
      const uint32_t d = pi / na, a = pi % na;
      const uint64_t *col = &lt.priv[(size_t)pi * BD];
#pragma unroll
      for (int aa = 0; aa < S::MA; ++aa) {
        if ((int)a == aa) {
          with_kind(S::kind(p, aa), [&](auto KC) {
            constexpr int K = decltype(KC)::value;
            uint64_t acc = col[part];
            for (int j = part + 8; j < BD; j += 8) acc = combine<K>(acc, col[j]);
#pragma unroll
            for (int off = 4; off >= 1; off >>= 1) acc = combine<K>(acc, __shfl_xor(acc, off, 8));
            if (part == 0) agg_merge_word(&lt.agg[aa * stride + lt.dslot[d]], K, acc);
          });
        }
      }
    }
    __syncthreads();
  }
  // merge the block's table into the global table
  const GTable t = *p.gt;
  const uint64_t gstr = t.cap + 1;
  for (uint32_t s = threadIdx.x; s < stride; s += BD) {
    const uint64_t w = lt.slot[s];
    const bool occ = s < cap ? w != kEmpty : lt.ctl[CTL_SPECIAL] != 0u;
    if (!occ) continue;
    const int64_t k1 = NK == 1 ? (int64_t)(s < cap ? w : kEmpty) : lt.k1[s];
    const int64_t k2 = NK == 1 ? 0 : lt.k2[s];
    const int64_t gs = g_find<NK>(t, key_hash<NK>(k1, k2), k1, k2);
    if (gs < 0) continue;
#pragma unroll
    for (int a = 0; a < S::MA; ++a)
      if (a < na) agg_merge_word(&t.agg[a * gstr + gs], S::kind(p, a), lt.agg[a * stride + s]);
  }
}

}  // namespace nut
