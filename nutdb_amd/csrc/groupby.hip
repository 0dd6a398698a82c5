// groupby.hip — fused  WHERE -> GROUP BY -> SUM/COUNT/MIN/MAX  (BASELINE configs 3, 4)
//
// Design:
//   * one streaming pass over the columns, 16 B per lane per load (two rows per lane,
//     four rows in flight per iteration), grid sized to the chip (blocks per CU from the
//     LDS footprint), grid-stride;
//   * every workgroup owns an open-addressing hash table in LDS: one 64-bit slot word,
//     then one 64-bit aggregate word per aggregate (SoA, so slots spread over banks);
//     rows update it with LDS atomics (ds_add_f64 / ds_add_u64 / ds_min,max_[ui]64);
//     f64 MIN/MAX use the IEEE total order mapped onto u64 so integer min/max apply;
//   * a block stops admitting NEW keys at 3/4 load; rows of keys it has not admitted go
//     to the global (HBM) table (exact for any G; fast while the hot keys fit on chip);
//   * at the end each block merges its occupied slots into the global table with
//     device-scope atomics.  Every cross-workgroup read of table words is a returning
//     atomic (memory side), never a plain or sc1 load that a stale L2 line could serve;
//   * single-key tables: the slot word IS the key (exact); the one key equal to the
//     empty marker lives in a dedicated extra slot.  Two-key tables: the key tuple is
//     written to an arena entry FIRST and the slot word {tag:32 | arena index:32} is
//     published by the claiming CAS, so a reader never waits for a half-written key.
// Algorithmic bytes: 8 B per referenced column per row (16 B/row config 3, 48 B/row Q1).
#include <string.h>

#include <algorithm>
#include <vector>

#include "common.hpp"

namespace nut {

enum AggKind : int32_t {
  AK_SUM_F64 = 0,
  AK_SUM_I64 = 1,  // also COUNT partials when merging
  AK_COUNT = 2,
  AK_MIN_F64 = 3,
  AK_MAX_F64 = 4,
  AK_MIN_I64 = 5,
  AK_MAX_I64 = 6,
};

constexpr uint64_t kEmpty2 = ~0ull;  // empty slot word of two-key tables

__host__ __device__ inline uint64_t agg_init(int kind) {
  switch (kind) {
    case AK_MIN_F64: return ~0ull;
    case AK_MAX_F64: return 0ull;
    case AK_MIN_I64: return 0x7FFFFFFFFFFFFFFFull;
    case AK_MAX_I64: return 0x8000000000000000ull;
    default: return 0ull;
  }
}

__device__ __forceinline__ int kind_at(uint32_t packed, int a) { return (int)((packed >> (4 * a)) & 15u); }

struct GTable {
  uint64_t *slot;    // [cap + 1]   slot `cap` = the empty-marker key (single-key tables)
  uint64_t *agg;     // [naggs][cap + 1]
  int64_t *ak1;      // [arena_cap] two-key tables: key tuples, written before publication
  int64_t *ak2;
  uint32_t *ctl;     // [0] claimed, [1] flags (1 overflow), [2] special used, [3] arena next
  uint64_t cap;      // power of two
  uint32_t limit;    // claims allowed before overflow is flagged
  uint32_t arena_cap;
  int log2cap;
  int naggs;
  uint32_t kinds;    // 4 bits per aggregate kind
};

struct AggArgs {
  uint64_t n;
  const int64_t *keys[2];
  const void *pred_col[NUT_MAX_PRED];
  uint64_t pred_k[NUT_MAX_PRED];  // constant bits
  int32_t pred_type[NUT_MAX_PRED];
  int32_t pred_op[NUT_MAX_PRED];
  const void *val_col[NUT_MAX_VALS];
  int32_t npred, nvals, naggs;
  uint32_t kinds;                 // 4 bits per aggregate kind
  int32_t expr[NUT_MAX_AGGS];
  int32_t arg[NUT_MAX_AGGS][3];
  uint32_t lds_cap;     // power of two, 0 = no LDS table
  uint32_t lds_limit;
  uint32_t lds_arena;
  int32_t lds_log2;
  int32_t vec;          // all columns 16-B aligned: vector loads
  const GTable *gt;     // device copy of the global table descriptor
};

__device__ __forceinline__ uint64_t pick(const uint64_t (&v)[NUT_MAX_VALS], int i) {
  return i == 0 ? v[0] : i == 1 ? v[1] : i == 2 ? v[2] : v[3];
}

// value word of aggregate a for one row (f64 bits or int64 bits)
__device__ __forceinline__ uint64_t agg_value(const AggArgs &p, int a, const uint64_t (&v)[NUT_MAX_VALS]) {
  const int e = p.expr[a];
  uint64_t x = pick(v, p.arg[a][0]);
  if (e == NUT_EX_COL) return x;
  double xa = as_f64(x), xb = as_f64(pick(v, p.arg[a][1]));
  double r;
  switch (e) {
    case NUT_EX_MUL: r = __dmul_rn(xa, xb); break;
    case NUT_EX_ADD: r = __dadd_rn(xa, xb); break;
    case NUT_EX_SUB: r = __dsub_rn(xa, xb); break;
    case NUT_EX_MUL_1M: r = __dmul_rn(xa, __dsub_rn(1.0, xb)); break;
    default: {
      double xc = as_f64(pick(v, p.arg[a][2]));
      r = __dmul_rn(__dmul_rn(xa, __dsub_rn(1.0, xb)), __dadd_rn(1.0, xc));
    }
  }
  return as_u64(r);
}

// atomic update of one aggregate word with one row's value (LDS or global)
__device__ __forceinline__ void agg_update(uint64_t *w, int kind, uint64_t x) {
  switch (kind) {
    case AK_SUM_F64: unsafeAtomicAdd((double *)w, as_f64(x)); break;
    case AK_SUM_I64: atomicAdd((unsigned long long *)w, (unsigned long long)x); break;
    case AK_COUNT: atomicAdd((unsigned long long *)w, 1ull); break;
    case AK_MIN_F64: atomicMin((unsigned long long *)w, (unsigned long long)f64_to_ord(x)); break;
    case AK_MAX_F64: atomicMax((unsigned long long *)w, (unsigned long long)f64_to_ord(x)); break;
    case AK_MIN_I64: atomicMin((long long *)w, (long long)x); break;
    default: atomicMax((long long *)w, (long long)x); break;
  }
}
// merge an already-aggregated word (COUNT merges by add; MIN/MAX f64 already ordered)
__device__ __forceinline__ void agg_merge_word(uint64_t *w, int kind, uint64_t x) {
  switch (kind) {
    case AK_SUM_F64: unsafeAtomicAdd((double *)w, as_f64(x)); break;
    case AK_SUM_I64:
    case AK_COUNT: atomicAdd((unsigned long long *)w, (unsigned long long)x); break;
    case AK_MIN_F64: atomicMin((unsigned long long *)w, (unsigned long long)x); break;
    case AK_MAX_F64: atomicMax((unsigned long long *)w, (unsigned long long)x); break;
    case AK_MIN_I64: atomicMin((long long *)w, (long long)x); break;
    default: atomicMax((long long *)w, (long long)x); break;
  }
}

// hash of the key tuple: single key -> the key itself is the slot word; two keys ->
// 64-bit mix (tag = high half, slot from multiply-shift)
template <int NK>
__device__ __forceinline__ uint64_t key_hash(int64_t k1, int64_t k2) {
  return NK == 1 ? (uint64_t)k1 : mix64((uint64_t)k1 ^ mix64((uint64_t)k2 + kGolden));
}

// ---- global table: find or claim the slot of a key tuple; -1 on overflow
template <int NK>
__device__ __forceinline__ int64_t g_find(const GTable &t, uint64_t h, int64_t k1, int64_t k2) {
  if (NK == 1 && h == kEmpty) {
    atomicOr(&t.ctl[2], 1u);
    return (int64_t)t.cap;
  }
  uint64_t s = slot_of(h, t.log2cap);
  const uint32_t tag = (uint32_t)(h >> 32);
  uint64_t word = kEmpty2;  // two-key: our published slot word once an arena entry is written
  for (uint64_t probe = 0; probe < t.cap; ++probe) {
    if (NK == 1) {
      uint64_t old = atomicCAS((unsigned long long *)&t.slot[s], (unsigned long long)kEmpty,
                               (unsigned long long)h);
      if (old == kEmpty) {
        if (atomicAdd(&t.ctl[0], 1u) >= t.limit) atomicOr(&t.ctl[1], 1u);
        return (int64_t)s;
      }
      if (old == h) return (int64_t)s;
    } else {
      uint64_t cur = rmw_load(&t.slot[s]);
      if (cur == kEmpty2) {
        if (word == kEmpty2) {
          uint32_t idx = atomicAdd(&t.ctl[3], 1u);
          if (idx >= t.arena_cap) {
            atomicOr(&t.ctl[1], 1u);
            return -1;
          }
          // publish the tuple at the memory side before the slot word can point at it
          atomicExch((unsigned long long *)&t.ak1[idx], (unsigned long long)k1);
          atomicExch((unsigned long long *)&t.ak2[idx], (unsigned long long)k2);
          word = ((uint64_t)tag << 32) | idx;
        }
        cur = __hip_atomic_compare_exchange_strong(&t.slot[s], &cur, word, __ATOMIC_RELEASE,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                  ? kEmpty2
                  : cur;
        if (cur == kEmpty2) {
          if (atomicAdd(&t.ctl[0], 1u) >= t.limit) atomicOr(&t.ctl[1], 1u);
          return (int64_t)s;
        }
      }
      if ((uint32_t)(cur >> 32) == tag) {
        uint32_t j = (uint32_t)cur;
        if ((int64_t)rmw_load((uint64_t *)&t.ak1[j]) == k1 && (int64_t)rmw_load((uint64_t *)&t.ak2[j]) == k2)
          return (int64_t)s;
      }
    }
    s = (s + 1) & (t.cap - 1);
  }
  atomicOr(&t.ctl[1], 1u);
  return -1;
}

// row-level fall-back for keys the block's LDS table did not admit (rare path; kept out
// of line so the streaming loop stays small)
template <int NK>
__device__ __noinline__ void g_row(const GTable *__restrict__ gtp, uint64_t h, int64_t k1, int64_t k2,
                                   uint64_t a0, uint64_t a1, uint64_t a2, uint64_t a3, uint64_t a4,
                                   uint64_t a5, uint64_t a6, uint64_t a7) {
  const GTable t = *gtp;
  int64_t gs = g_find<NK>(t, h, k1, k2);
  if (gs < 0) return;
  const uint64_t stride = t.cap + 1;
  const uint64_t av[8] = {a0, a1, a2, a3, a4, a5, a6, a7};
#pragma unroll
  for (int a = 0; a < NUT_MAX_AGGS; ++a)
    if (a < t.naggs) agg_update(&t.agg[a * stride + gs], kind_at(t.kinds, a), av[a]);
}

// LDS table view (dynamic shared memory, carved in this order, 16-B aligned)
struct LTable {
  uint64_t *slot;   // [cap + 1]
  uint64_t *agg;    // [naggs][cap + 1]
  int64_t *ak1;     // [arena] (NK == 2)
  int64_t *ak2;
  uint32_t *ctl;    // [0] claimed, [1] special used, [2] arena next
};

template <int NK>
__device__ __forceinline__ int32_t l_find(const LTable &t, const AggArgs &p, uint64_t h, int64_t k1, int64_t k2) {
  const uint32_t cap = p.lds_cap;
  if (NK == 1 && h == kEmpty) {
    t.ctl[1] = 1u;
    return (int32_t)cap;
  }
  uint32_t s = slot_of(h, p.lds_log2);
  const uint32_t tag = (uint32_t)(h >> 32);
  uint64_t word = kEmpty2;
  const uint64_t empty = NK == 1 ? kEmpty : kEmpty2;
  for (uint32_t probe = 0; probe < cap; ++probe) {
    uint64_t cur = t.slot[s];
    bool won = false;
    if (cur == empty) {
      if (*(volatile uint32_t *)&t.ctl[0] >= p.lds_limit) return -1;  // closed to new keys
      if (NK == 1) {
        cur = atomicCAS((unsigned long long *)&t.slot[s], (unsigned long long)kEmpty, (unsigned long long)h);
        won = cur == kEmpty;
      } else {
        if (word == kEmpty2) {
          uint32_t idx = atomicAdd(&t.ctl[2], 1u);
          if (idx >= p.lds_arena) return -1;
          t.ak1[idx] = k1;
          t.ak2[idx] = k2;
          word = ((uint64_t)tag << 32) | idx;
        }
        // release: the arena stores are performed before the slot word is visible
        won = __hip_atomic_compare_exchange_strong(&t.slot[s], &cur, word, __ATOMIC_RELEASE, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (won) atomicAdd(&t.ctl[0], 1u);
    }
    if (won) return (int32_t)s;
    if (NK == 1) {
      if (cur == h) return (int32_t)s;
    } else if ((uint32_t)(cur >> 32) == tag) {
      uint32_t j = (uint32_t)cur;
      if (t.ak1[j] == k1 && t.ak2[j] == k2) return (int32_t)s;
    }
    s = (s + 1) & (cap - 1);
  }
  return -1;
}

template <int NK>
__device__ __forceinline__ void process_row(const AggArgs &p, const LTable &lt, int64_t k1, int64_t k2,
                                            const uint64_t (&v)[NUT_MAX_VALS]) {
  const uint64_t h = key_hash<NK>(k1, k2);
  uint64_t av[NUT_MAX_AGGS];
#pragma unroll
  for (int a = 0; a < NUT_MAX_AGGS; ++a)
    av[a] = (a < p.naggs && kind_at(p.kinds, a) != AK_COUNT) ? agg_value(p, a, v) : 0;
  const int32_t ls = p.lds_cap ? l_find<NK>(lt, p, h, k1, k2) : -1;
  if (ls >= 0) {
    const uint32_t stride = p.lds_cap + 1;
    // compile-time aggregate indices: a runtime index into the kernel-argument
    // struct would spill it to scratch
#pragma unroll
    for (int a = 0; a < NUT_MAX_AGGS; ++a)
      if (a < p.naggs) agg_update(&lt.agg[a * stride + ls], kind_at(p.kinds, a), av[a]);
  } else {
    g_row<NK>(p.gt, h, k1, k2, av[0], av[1], av[2], av[3], av[4], av[5], av[6], av[7]);
  }
}

__device__ __forceinline__ bool row_pass(const AggArgs &p, const uint64_t (&pv)[NUT_MAX_PRED]) {
  bool ok = true;
#pragma unroll
  for (int t = 0; t < NUT_MAX_PRED; ++t) {
    if (t < p.npred) {
      bool r = p.pred_type[t] == NUT_T_I64 ? cmp_i64((int64_t)pv[t], p.pred_op[t], (int64_t)p.pred_k[t])
                                            : cmp_f64(as_f64(pv[t]), p.pred_op[t], as_f64(p.pred_k[t]));
      ok = ok && r;
    }
  }
  return ok;
}

__device__ __forceinline__ u64x2 ld2(const void *col, uint64_t i, bool vec) {
  const uint64_t *c = (const uint64_t *)col + i;
  if (vec) return *reinterpret_cast<const u64x2 *>(c);  // uniform branch: 16-B aligned columns
  u64x2 r;
  r.x = c[0];
  r.y = c[1];
  return r;
}
__device__ __forceinline__ u64x2 ld2_tail(const void *col, uint64_t i, uint64_t n) {
  const uint64_t *c = (const uint64_t *)col;
  u64x2 r;
  r.x = i < n ? c[i] : 0;
  r.y = i + 1 < n ? c[i + 1] : 0;
  return r;
}

// the columns of one pair of rows (one 16-B load per referenced column)
template <int NK>
struct Pair {
  u64x2 k1, k2, pv[NUT_MAX_PRED], vv[NUT_MAX_VALS];
};

template <int NK, bool TAIL>
__device__ __forceinline__ void load_pair(const AggArgs &p, uint64_t i, Pair<NK> &x) {
#pragma unroll
  for (int t = 0; t < NUT_MAX_PRED; ++t)
    if (t < p.npred) x.pv[t] = TAIL ? ld2_tail(p.pred_col[t], i, p.n) : ld2(p.pred_col[t], i, p.vec);
  x.k1 = TAIL ? ld2_tail(p.keys[0], i, p.n) : ld2(p.keys[0], i, p.vec);
  if (NK == 2) x.k2 = TAIL ? ld2_tail(p.keys[1], i, p.n) : ld2(p.keys[1], i, p.vec);
#pragma unroll
  for (int c = 0; c < NUT_MAX_VALS; ++c)
    if (c < p.nvals) x.vv[c] = TAIL ? ld2_tail(p.val_col[c], i, p.n) : ld2(p.val_col[c], i, p.vec);
}

template <int NK, bool TAIL>
__device__ __forceinline__ void consume_pair(const AggArgs &p, const LTable &lt, uint64_t i, const Pair<NK> &x) {
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint64_t pr[NUT_MAX_PRED], vr[NUT_MAX_VALS];
#pragma unroll
    for (int t = 0; t < NUT_MAX_PRED; ++t) pr[t] = t < p.npred ? (r ? x.pv[t].y : x.pv[t].x) : 0;
#pragma unroll
    for (int c = 0; c < NUT_MAX_VALS; ++c) vr[c] = c < p.nvals ? (r ? x.vv[c].y : x.vv[c].x) : 0;
    const bool ok = row_pass(p, pr) && (!TAIL || i + r < p.n);
    if (ok)
      process_row<NK>(p, lt, (int64_t)(r ? x.k1.y : x.k1.x), NK == 2 ? (int64_t)(r ? x.k2.y : x.k2.x) : 0, vr);
  }
}

template <int NK>
__global__ __launch_bounds__(512) void agg_kernel(AggArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const uint32_t cap = p.lds_cap;
  const uint32_t stride = cap + 1;
  LTable lt;
  lt.slot = smem;
  lt.agg = lt.slot + stride;
  lt.ak1 = (int64_t *)(lt.agg + (size_t)p.naggs * stride);
  lt.ak2 = lt.ak1 + (NK == 2 ? p.lds_arena : 0);
  lt.ctl = (uint32_t *)(lt.ak2 + (NK == 2 ? p.lds_arena : 0));

  if (cap) {
    const uint64_t empty = NK == 1 ? kEmpty : kEmpty2;
    for (uint32_t s = threadIdx.x; s < stride; s += blockDim.x) {
      lt.slot[s] = empty;
#pragma unroll
      for (int a = 0; a < NUT_MAX_AGGS; ++a)
        if (a < p.naggs) lt.agg[a * stride + s] = agg_init(kind_at(p.kinds, a));
    }
    if (threadIdx.x < 4) lt.ctl[threadIdx.x] = 0;
    __syncthreads();
  }

  // grid-stride over pairs of rows, two pairs (4 rows, 2 loads per column) in flight
  const uint64_t npairs = (p.n + 1) / 2;
  const uint64_t full_pairs = p.n / 2;
  const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; q + gstride < full_pairs; q += 2 * gstride) {
    Pair<NK> a, b;
    load_pair<NK, false>(p, 2 * q, a);
    load_pair<NK, false>(p, 2 * (q + gstride), b);
    consume_pair<NK, false>(p, lt, 2 * q, a);
    consume_pair<NK, false>(p, lt, 2 * (q + gstride), b);
  }
  for (; q < npairs; q += gstride) {
    Pair<NK> a;
    load_pair<NK, true>(p, 2 * q, a);
    consume_pair<NK, true>(p, lt, 2 * q, a);
  }

  if (!cap) return;
  __syncthreads();
  // merge the block's table into the global table
  const GTable t = *p.gt;
  const uint64_t gstr = t.cap + 1;
  for (uint32_t s = threadIdx.x; s < stride; s += blockDim.x) {
    const uint64_t w = lt.slot[s];
    bool occ;
    int64_t k1, k2 = 0;
    uint64_t h;
    if (NK == 1) {
      occ = s < cap ? w != kEmpty : lt.ctl[1] != 0u;
      h = s < cap ? w : kEmpty;
      k1 = (int64_t)h;
    } else {
      occ = s < cap && w != kEmpty2;
      uint32_t j = (uint32_t)w;
      k1 = occ ? lt.ak1[j] : 0;
      k2 = occ ? lt.ak2[j] : 0;
      h = key_hash<2>(k1, k2);
    }
    if (!occ) continue;
    int64_t gs = g_find<NK>(t, h, k1, k2);
    if (gs < 0) continue;
#pragma unroll
    for (int a = 0; a < NUT_MAX_AGGS; ++a)
      if (a < p.naggs) agg_merge_word(&t.agg[a * gstr + gs], kind_at(p.kinds, a), lt.agg[a * stride + s]);
  }
}

// ---- global table init / compaction / partition / rehash
__global__ void gtable_init_kernel(const GTable *__restrict__ gtp, int nk) {
  const GTable t = *gtp;
  const uint64_t stride = t.cap + 1;
  const uint64_t empty = nk == 1 ? kEmpty : kEmpty2;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < stride;
       s += (uint64_t)gridDim.x * blockDim.x) {
    t.slot[s] = empty;
    for (int a = 0; a < t.naggs; ++a) t.agg[a * stride + s] = agg_init(kind_at(t.kinds, a));
  }
}

// occupied slot s -> (k1, k2); false if empty
__device__ __forceinline__ bool slot_keys(const GTable &t, int nk, uint64_t s, uint64_t &k1, uint64_t &k2) {
  if (nk == 1) {
    if (s == t.cap) {
      k1 = kEmpty;
      k2 = 0;
      return t.ctl[2] != 0u;
    }
    k1 = t.slot[s];
    k2 = 0;
    return k1 != kEmpty;
  }
  if (s == t.cap) return false;
  uint64_t w = t.slot[s];
  if (w == kEmpty2) return false;
  k1 = (uint64_t)t.ak1[(uint32_t)w];
  k2 = (uint64_t)t.ak2[(uint32_t)w];
  return true;
}

// dense column-major copy of the occupied slots; owner partitioning optional
__global__ void gtable_compact_kernel(const GTable *__restrict__ gtp, int nk, uint64_t *__restrict__ out,
                                      uint64_t out_cap, unsigned long long *__restrict__ cursors, int nparts,
                                      const uint64_t *__restrict__ seg_base) {
  const GTable t = *gtp;
  const uint64_t stride = t.cap + 1;
  const int w = nk + t.naggs;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < stride;
       s += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k1, k2;
    if (!slot_keys(t, nk, s, k1, k2)) continue;
    int part = nparts > 1 ? (int)(owner_hash(k1, k2, nk) % (uint64_t)nparts) : 0;
    uint64_t pos = atomicAdd(&cursors[part], 1ull);
    // segment `part` starts at word w*seg_base[part]; each of its columns has seg_n rows
    uint64_t seg_n = nparts > 1 ? seg_base[nparts + part] : out_cap;
    uint64_t *seg = out + (nparts > 1 ? (uint64_t)w * seg_base[part] : 0);
    seg[pos] = k1;
    if (nk == 2) seg[seg_n + pos] = k2;
    for (int a = 0; a < t.naggs; ++a) {
      uint64_t x = t.agg[a * stride + s];
      int kind = kind_at(t.kinds, a);
      if (kind == AK_MIN_F64 || kind == AK_MAX_F64) x = ord_to_f64(x);
      seg[(uint64_t)(nk + a) * seg_n + pos] = x;
    }
  }
}

__global__ void gtable_owner_count_kernel(const GTable *__restrict__ gtp, int nk, int nparts,
                                          unsigned long long *counts) {
  const GTable t = *gtp;
  const uint64_t stride = t.cap + 1;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < stride;
       s += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k1, k2;
    if (!slot_keys(t, nk, s, k1, k2)) continue;
    atomicAdd(&counts[owner_hash(k1, k2, nk) % (uint64_t)nparts], 1ull);
  }
}

__global__ void rehash_kernel(const GTable *__restrict__ srcp, const GTable *__restrict__ dstp, int nk) {
  const GTable src = *srcp, dst = *dstp;
  const uint64_t stride = src.cap + 1;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < stride;
       s += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k1, k2;
    if (!slot_keys(src, nk, s, k1, k2)) continue;
    int64_t d = nk == 1 ? g_find<1>(dst, key_hash<1>((int64_t)k1, 0), (int64_t)k1, 0)
                        : g_find<2>(dst, key_hash<2>((int64_t)k1, (int64_t)k2), (int64_t)k1, (int64_t)k2);
    if (d < 0) continue;
    for (int a = 0; a < src.naggs; ++a)
      agg_merge_word(&dst.agg[a * (dst.cap + 1) + d], kind_at(src.kinds, a), src.agg[a * stride + s]);
  }
}

}  // namespace nut

// ============================================================== host side
using namespace nut;

struct nut_groups {
  nut_ctx *ctx = nullptr;
  int nk = 1, naggs = 0;
  int32_t kinds[NUT_MAX_AGGS] = {0};
  GTable gt{};                     // host copy of the descriptor
  GTable *dev_gt = nullptr;        // device copy (inside mem)
  void *mem = nullptr;             // table allocation
  size_t mem_bytes = 0;
  unsigned long long *dev_cursors = nullptr;  // [64] inside mem
  uint64_t *dev_segbase = nullptr;            // [2*64] inside mem
};

namespace {

int ilog2(uint64_t v) {
  int r = 0;
  while ((1ull << r) < v) ++r;
  return r;
}

uint32_t pack_kinds(const int32_t *k, int n) {
  uint32_t p = 0;
  for (int a = 0; a < n; ++a) p |= (uint32_t)(k[a] & 15) << (4 * a);
  return p;
}

nut_status validate(const nut_agg_spec *s) {
  if (!s) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: spec is NULL");
  if (s->nkeys < 1 || s->nkeys > 2) return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: 1 or 2 key columns supported");
  if (s->npred < 0 || s->npred > NUT_MAX_PRED) return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: too many predicate terms");
  if (s->nvals < 0 || s->nvals > NUT_MAX_VALS) return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: too many value columns");
  if (s->naggs < 0 || s->naggs > NUT_MAX_AGGS) return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: too many aggregates");
  if (s->n) {
    for (int k = 0; k < s->nkeys; ++k)
      if (!s->keys[k]) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: NULL key column");
    for (int t = 0; t < s->npred; ++t) {
      if (!s->pred_col[t]) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: NULL predicate column");
      if (s->pred_op[t] < NUT_LT || s->pred_op[t] > NUT_NE) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad cmp op");
      if (s->pred_type[t] != NUT_T_I64 && s->pred_type[t] != NUT_T_F64)
        return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad predicate type");
    }
    for (int c = 0; c < s->nvals; ++c)
      if (!s->val_col[c]) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: NULL value column");
  }
  for (int a = 0; a < s->naggs; ++a) {
    int op = s->agg_op[a];
    if (op < NUT_AGG_SUM || op > NUT_AGG_MAX) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad aggregate op");
    if (op == NUT_AGG_COUNT) continue;
    int e = s->agg_expr[a];
    if (e < NUT_EX_COL || e > NUT_EX_MUL_1M_1P) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad expression");
    int nargs = e == NUT_EX_COL ? 1 : e == NUT_EX_MUL_1M_1P ? 3 : 2;
    for (int j = 0; j < nargs; ++j) {
      int v = s->agg_arg[a][j];
      if (v < 0 || v >= s->nvals) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: expression argument out of range");
      if (e != NUT_EX_COL && s->val_type[v] != NUT_T_F64)
        return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: arithmetic expressions need f64 columns");
    }
  }
  return NUT_OK;
}

int32_t kind_of(const nut_agg_spec *s, int a) {
  int op = s->agg_op[a];
  if (op == NUT_AGG_COUNT) return AK_COUNT;
  bool i64 = s->agg_expr[a] == NUT_EX_COL && s->val_type[s->agg_arg[a][0]] == NUT_T_I64;
  switch (op) {
    case NUT_AGG_SUM: return i64 ? AK_SUM_I64 : AK_SUM_F64;
    case NUT_AGG_MIN: return i64 ? AK_MIN_I64 : AK_MIN_F64;
    default: return i64 ? AK_MAX_I64 : AK_MAX_F64;
  }
}

// LDS bytes of a table with `cap` slots (+1 special); two-key tables add a key arena
// of `cap` tuples (3/4 of it holds admitted keys, the rest absorbs lost claim races)
size_t lds_bytes(uint32_t cap, int nk, int naggs) {
  if (cap == 0) return 0;
  size_t stride = cap + 1;
  size_t b = stride * 8 * (1 + naggs);
  if (nk == 2) b += (size_t)cap * 16;
  b += 16;
  return (b + 15) & ~size_t(15);
}

// (re)allocate the global table for `cap` slots and initialise it on the stream
nut_status alloc_table(nut_groups *g, uint64_t cap) {
  const uint64_t stride = cap + 1;
  // two-key arena: one entry per claimable slot plus slack for claim races lost by
  // concurrent inserters of the same key (each loser leaks at most one entry)
  const uint64_t arena = g->nk == 2 ? cap + 65536 : 0;
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  size_t o_slot = carve(stride * 8);
  size_t o_agg = carve(stride * 8 * (size_t)std::max(g->naggs, 1));
  size_t o_a1 = carve(arena * 8 + 8);
  size_t o_a2 = carve(arena * 8 + 8);
  size_t o_ctl = carve(64);
  size_t o_gt = carve(sizeof(GTable));
  size_t o_cur = carve(64 * 8);
  size_t o_seg = carve(128 * 8);
  if (!(g->mem && g->mem_bytes >= off)) {
    if (g->mem) (void)hipFree(g->mem);
    g->mem = nullptr;
    NUT_HIP(hipMalloc(&g->mem, off));
    g->mem_bytes = off;
  }
  char *b = (char *)g->mem;
  GTable &t = g->gt;
  t.slot = (uint64_t *)(b + o_slot);
  t.agg = (uint64_t *)(b + o_agg);
  t.ak1 = (int64_t *)(b + o_a1);
  t.ak2 = (int64_t *)(b + o_a2);
  t.ctl = (uint32_t *)(b + o_ctl);
  t.cap = cap;
  t.log2cap = ilog2(cap);
  t.limit = (uint32_t)std::min<uint64_t>(cap - cap / 4, 0xFFFFFFF0ull);
  t.arena_cap = (uint32_t)std::min<uint64_t>(arena, 0xFFFFFFF0ull);
  t.naggs = g->naggs;
  t.kinds = pack_kinds(g->kinds, g->naggs);
  g->dev_gt = (GTable *)(b + o_gt);
  g->dev_cursors = (unsigned long long *)(b + o_cur);
  g->dev_segbase = (uint64_t *)(b + o_seg);
  hipStream_t st = g->ctx->stream;
  NUT_HIP(hipMemsetAsync(t.ctl, 0, 64, st));
  NUT_HIP(hipMemcpyAsync(g->dev_gt, &g->gt, sizeof(GTable), hipMemcpyHostToDevice, st));
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)g->ctx->num_cus * 8);
  hipLaunchKernelGGL(gtable_init_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const GTable *)g->dev_gt, g->nk);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

nut_status read_ctl(nut_groups *g, uint32_t *ctl4) {
  nut_ctx *c = g->ctx;
  NUT_HIP(hipMemcpyAsync(c->host_pinned, g->gt.ctl, 16, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  memcpy(ctl4, c->host_pinned, 16);
  return NUT_OK;
}

// launch the streaming aggregation of spec's rows into g's table.  `kinds` are the
// per-row update kinds (COUNT partials are merged as integer sums).
nut_status launch_agg(nut_groups *g, const nut_agg_spec *s, uint64_t group_hint, const int32_t *kinds) {
  nut_ctx *c = g->ctx;
  if (s->n == 0) return NUT_OK;
  AggArgs a;
  memset(&a, 0, sizeof(a));
  a.n = s->n;
  a.keys[0] = s->keys[0];
  a.keys[1] = s->nkeys == 2 ? s->keys[1] : s->keys[0];
  a.npred = s->npred;
  for (int t = 0; t < s->npred; ++t) {
    a.pred_col[t] = s->pred_col[t];
    a.pred_type[t] = s->pred_type[t];
    a.pred_op[t] = s->pred_op[t];
    if (s->pred_type[t] == NUT_T_I64) a.pred_k[t] = (uint64_t)s->pred_i64[t];
    else memcpy(&a.pred_k[t], &s->pred_f64[t], 8);
  }
  a.nvals = s->nvals;
  for (int v = 0; v < s->nvals; ++v) a.val_col[v] = s->val_col[v];
  a.naggs = s->naggs;
  a.kinds = pack_kinds(kinds, s->naggs);
  for (int i = 0; i < s->naggs; ++i) {
    a.expr[i] = s->agg_op[i] == NUT_AGG_COUNT ? NUT_EX_COL : s->agg_expr[i];
    for (int j = 0; j < 3; ++j) a.arg[i][j] = s->agg_op[i] == NUT_AGG_COUNT ? 0 : s->agg_arg[i][j];
  }
  // all columns must be 16-B aligned for the vector loads
  auto misaligned = [](const void *ptr) { return ((uintptr_t)ptr & 15) != 0; };
  bool bad = misaligned(a.keys[0]) || misaligned(a.keys[1]);
  for (int t = 0; t < a.npred; ++t) bad |= misaligned(a.pred_col[t]);
  for (int v = 0; v < a.nvals; ++v) bad |= misaligned(a.val_col[v]);
  a.vec = bad ? 0 : 1;  // 8-B aligned columns (e.g. slices) take two 8-B loads per pair

  // on-chip table: 2x the expected groups within the LDS budget
  const size_t lds_max = 160 * 1024;
  uint64_t want = group_hint ? 2 * group_hint : 4096;
  uint32_t lcap = 64;
  while (lcap < want && lds_bytes(lcap * 2, g->nk, g->naggs) <= lds_max) lcap *= 2;
  if (group_hint > 8ull * lcap) lcap = 0;  // hot keys cannot fit on chip: straight to HBM
  a.lds_cap = lcap;
  a.lds_limit = lcap - lcap / 4;
  a.lds_arena = g->nk == 2 ? lcap : 0;
  a.lds_log2 = lcap ? ilog2(lcap) : 0;
  a.gt = g->dev_gt;
  size_t lb = lds_bytes(lcap, g->nk, g->naggs);
  const int threads = 512;
  int blocks_per_cu = lb ? (int)std::max<size_t>(1, std::min<size_t>(4, lds_max / lb)) : 4;
  uint64_t pairs = (s->n + 1) / 2;
  uint64_t blocks = std::min<uint64_t>((uint64_t)c->num_cus * blocks_per_cu, (pairs + threads - 1) / threads);
  if (blocks == 0) blocks = 1;
  static bool attr_set = false;
  if (!attr_set) {
    NUT_HIP(hipFuncSetAttribute((const void *)agg_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
    NUT_HIP(hipFuncSetAttribute((const void *)agg_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
    attr_set = true;
  }
  c->timer.begin(c->stream, NUT_KERNEL_AGGREGATE);
  if (g->nk == 1)
    hipLaunchKernelGGL(agg_kernel<1>, dim3((unsigned)blocks), dim3(threads), lb, c->stream, a);
  else
    hipLaunchKernelGGL(agg_kernel<2>, dim3((unsigned)blocks), dim3(threads), lb, c->stream, a);
  c->timer.end(c->stream);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

uint64_t table_cap_for(uint64_t groups) {
  uint64_t cap = 1024;
  while (cap < 2 * groups) cap *= 2;
  return cap;
}

// grow the table (rehash existing groups) so that `extra` more groups fit
nut_status ensure_room(nut_groups *g, uint64_t extra) {
  uint32_t ctl[4];
  nut_status st = read_ctl(g, ctl);
  if (st) return st;
  uint64_t need = (uint64_t)ctl[0] + extra + 1;
  if (need <= g->gt.limit && (g->nk == 1 || (uint64_t)ctl[3] + extra <= g->gt.arena_cap)) return NUT_OK;
  nut_groups fresh;
  fresh.ctx = g->ctx;
  fresh.nk = g->nk;
  fresh.naggs = g->naggs;
  memcpy(fresh.kinds, g->kinds, sizeof(g->kinds));
  st = alloc_table(&fresh, table_cap_for(need));
  if (st) return st;
  nut_ctx *c = g->ctx;
  uint64_t stride = g->gt.cap + 1;
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)c->num_cus * 8);
  hipLaunchKernelGGL(rehash_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, (const GTable *)g->dev_gt,
                     (const GTable *)fresh.dev_gt, g->nk);
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipStreamSynchronize(c->stream));
  (void)hipFree(g->mem);
  g->mem = fresh.mem;
  g->mem_bytes = fresh.mem_bytes;
  g->gt = fresh.gt;
  g->dev_gt = fresh.dev_gt;
  g->dev_cursors = fresh.dev_cursors;
  g->dev_segbase = fresh.dev_segbase;
  fresh.mem = nullptr;
  return NUT_OK;
}

}  // namespace

extern "C" {

nut_status nut_groupby(nut_ctx *c, const nut_agg_spec *s, uint64_t group_hint, nut_groups **out) {
  if (!c || !out) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: NULL argument");
  *out = nullptr;
  nut_status st = validate(s);
  if (st) return st;
  DeviceGuard dg(c->device);
  nut_groups *g = new nut_groups();
  g->ctx = c;
  g->nk = s->nkeys;
  g->naggs = s->naggs;
  for (int a = 0; a < s->naggs; ++a) g->kinds[a] = kind_of(s, a);
  uint64_t cap = table_cap_for(group_hint ? group_hint : 8192);
  for (int attempt = 0;; ++attempt) {
    st = alloc_table(g, cap);
    if (!st) st = launch_agg(g, s, group_hint, g->kinds);
    uint32_t ctl[4] = {0, 0, 0, 0};
    if (!st) st = read_ctl(g, ctl);
    if (st) {
      nut_groups_free(g);
      return st;
    }
    if (!(ctl[1] & 1u)) break;
    // more groups than the table admits: retry with a larger table
    if (cap >= (1ull << 34) || attempt > 12) {
      nut_groups_free(g);
      return fail(NUT_ERR_OOM, "nut_groupby: group table would exceed device memory");
    }
    cap *= 4;
    group_hint = std::max<uint64_t>(group_hint, ctl[0]);
  }
  *out = g;
  return NUT_OK;
}

nut_status nut_groupby_accumulate(nut_ctx *c, const nut_agg_spec *s, nut_groups *g) {
  if (!c || !g) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_accumulate: NULL argument");
  nut_status st = validate(s);
  if (st) return st;
  if (s->nkeys != g->nk || s->naggs != g->naggs)
    return fail(NUT_ERR_INVALID_ARG, "nut_groupby_accumulate: spec shape differs from the result");
  int32_t kinds[NUT_MAX_AGGS];
  for (int a = 0; a < s->naggs; ++a) {
    int32_t k = kind_of(s, a);
    bool same = k == g->kinds[a] || (g->kinds[a] == AK_COUNT && k == AK_SUM_I64);
    if (!same) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_accumulate: aggregate kinds differ");
    kinds[a] = g->kinds[a] == AK_COUNT ? AK_SUM_I64 : k;  // COUNT partials merge by addition
  }
  DeviceGuard dg(c->device);
  g->ctx = c;
  st = ensure_room(g, s->n);
  if (st) return st;
  st = launch_agg(g, s, s->n, kinds);
  if (st) return st;
  uint32_t ctl[4];
  st = read_ctl(g, ctl);
  if (st) return st;
  if (ctl[1]) return fail(NUT_ERR_OOM, "nut_groupby_accumulate: table overflow");
  return NUT_OK;
}

nut_status nut_groups_size(nut_groups *g, uint64_t *n) {
  if (!g || !n) return fail(NUT_ERR_INVALID_ARG, "nut_groups_size: NULL argument");
  DeviceGuard dg(g->ctx->device);
  uint32_t ctl[4];
  nut_status st = read_ctl(g, ctl);
  if (st) return st;
  *n = (uint64_t)ctl[0] + (g->nk == 1 && ctl[2] ? 1 : 0);
  return NUT_OK;
}

nut_status nut_groups_to_device(nut_groups *g, uint64_t *out, uint64_t cap) {
  if (!g) return fail(NUT_ERR_INVALID_ARG, "nut_groups_to_device: NULL argument");
  uint64_t n;
  nut_status st = nut_groups_size(g, &n);
  if (st) return st;
  if (n > cap)
    return fail(NUT_ERR_CAPACITY, "nut_groups_to_device: capacity " + std::to_string(cap) + " < " +
                                      std::to_string(n) + " groups");
  if (n == 0) return NUT_OK;
  if (!out) return fail(NUT_ERR_INVALID_ARG, "nut_groups_to_device: NULL output");
  nut_ctx *c = g->ctx;
  DeviceGuard dg(c->device);
  NUT_HIP(hipMemsetAsync(g->dev_cursors, 0, 64 * 8, c->stream));
  uint64_t stride = g->gt.cap + 1;
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)c->num_cus * 8);
  hipLaunchKernelGGL(gtable_compact_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream,
                     (const GTable *)g->dev_gt, g->nk, out, n, g->dev_cursors, 1, (const uint64_t *)nullptr);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

nut_status nut_groups_partition(nut_groups *g, int nparts, uint64_t *out, uint64_t cap, uint64_t *counts) {
  if (!g || !counts || nparts < 1 || nparts > 64) return fail(NUT_ERR_INVALID_ARG, "nut_groups_partition: bad argument");
  nut_ctx *c = g->ctx;
  DeviceGuard dg(c->device);
  uint64_t n;
  nut_status st = nut_groups_size(g, &n);
  if (st) return st;
  if (n > cap) return fail(NUT_ERR_CAPACITY, "nut_groups_partition: capacity too small");
  if (nparts == 1) {
    counts[0] = n;
    return nut_groups_to_device(g, out, cap);
  }
  uint64_t stride = g->gt.cap + 1;
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)c->num_cus * 8);
  NUT_HIP(hipMemsetAsync(g->dev_cursors, 0, 64 * 8, c->stream));
  hipLaunchKernelGGL(gtable_owner_count_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream,
                     (const GTable *)g->dev_gt, g->nk, nparts, g->dev_cursors);
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipMemcpyAsync(c->host_pinned, g->dev_cursors, 8 * nparts, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  uint64_t seg[128];
  uint64_t run = 0;
  for (int p = 0; p < nparts; ++p) {
    counts[p] = c->host_pinned[p];
    seg[p] = run;
    seg[nparts + p] = counts[p];
    run += counts[p];
  }
  if (run == 0) return NUT_OK;
  if (!out) return fail(NUT_ERR_INVALID_ARG, "nut_groups_partition: NULL output");
  NUT_HIP(hipMemcpyAsync(g->dev_segbase, seg, 16 * nparts, hipMemcpyHostToDevice, c->stream));
  NUT_HIP(hipMemsetAsync(g->dev_cursors, 0, 64 * 8, c->stream));
  hipLaunchKernelGGL(gtable_compact_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream,
                     (const GTable *)g->dev_gt, g->nk, out, run, g->dev_cursors, nparts,
                     (const uint64_t *)g->dev_segbase);
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipStreamSynchronize(c->stream));
  return NUT_OK;
}

nut_status nut_groups_to_host(nut_groups *g, int64_t *keys, uint64_t *aggs, uint64_t cap) {
  if (!g) return fail(NUT_ERR_INVALID_ARG, "nut_groups_to_host: NULL argument");
  uint64_t n;
  nut_status st = nut_groups_size(g, &n);
  if (st) return st;
  if (n > cap)
    return fail(NUT_ERR_CAPACITY, "nut_groups_to_host: capacity " + std::to_string(cap) + " < " +
                                      std::to_string(n) + " groups");
  if (n == 0) return NUT_OK;
  if (!keys || (g->naggs && !aggs)) return fail(NUT_ERR_INVALID_ARG, "nut_groups_to_host: NULL output");
  nut_ctx *c = g->ctx;
  DeviceGuard dg(c->device);
  const int w = g->nk + g->naggs;
  uint64_t *dev = nullptr;
  NUT_HIP(hipMallocAsync((void **)&dev, (size_t)w * n * 8, c->stream));
  st = nut_groups_to_device(g, dev, n);
  std::vector<uint64_t> h((size_t)w * n);
  if (!st) {
    hipError_t e = hipMemcpyAsync(h.data(), dev, (size_t)w * n * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) st = hip_fail(e, "nut_groups_to_host copy");
  }
  (void)hipFreeAsync(dev, c->stream);
  if (st) return st;
  std::vector<uint64_t> order(n);
  for (uint64_t i = 0; i < n; ++i) order[i] = i;
  const int nk = g->nk;
  std::sort(order.begin(), order.end(), [&](uint64_t x, uint64_t y) {
    int64_t a0 = (int64_t)h[x], b0 = (int64_t)h[y];
    if (a0 != b0) return a0 < b0;
    if (nk == 2) return (int64_t)h[n + x] < (int64_t)h[n + y];
    return false;
  });
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t src = order[i];
    for (int j = 0; j < nk; ++j) keys[i * nk + j] = (int64_t)h[(size_t)j * n + src];
    for (int a = 0; a < g->naggs; ++a) aggs[i * g->naggs + a] = h[(size_t)(nk + a) * n + src];
  }
  return NUT_OK;
}

void nut_groups_free(nut_groups *g) {
  if (!g) return;
  if (g->mem) {
    DeviceGuard dg(g->ctx->device);
    (void)hipStreamSynchronize(g->ctx->stream);
    (void)hipFree(g->mem);
  }
  delete g;
}

nut_status nut_groupby_i64_f64(nut_ctx *c, const int64_t *key, const double *val, uint64_t n, uint32_t mask,
                               uint64_t group_hint, nut_groups **out) {
  nut_agg_spec s;
  memset(&s, 0, sizeof(s));
  s.n = n;
  s.nkeys = 1;
  s.keys[0] = key;
  s.nvals = 1;
  s.val_col[0] = val;
  s.val_type[0] = NUT_T_F64;
  const int ops[4] = {NUT_AGG_SUM, NUT_AGG_COUNT, NUT_AGG_MIN, NUT_AGG_MAX};
  for (int b = 0; b < 4; ++b)
    if (mask & (1u << b)) {
      s.agg_op[s.naggs] = ops[b];
      s.agg_expr[s.naggs] = NUT_EX_COL;
      ++s.naggs;
    }
  if (s.naggs == 0) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_i64_f64: empty aggregate mask");
  return nut_groupby(c, &s, group_hint, out);
}

nut_status nut_q1(nut_ctx *c, const int64_t *shipdate, const int64_t *returnflag, const int64_t *linestatus,
                  const double *qty, const double *price, const double *disc, uint64_t n, int64_t date_k,
                  nut_groups **out) {
  nut_agg_spec s;
  memset(&s, 0, sizeof(s));
  s.n = n;
  s.nkeys = 2;
  s.keys[0] = returnflag;
  s.keys[1] = linestatus;
  s.npred = 1;
  s.pred_col[0] = shipdate;
  s.pred_type[0] = NUT_T_I64;
  s.pred_op[0] = NUT_LE;
  s.pred_i64[0] = date_k;
  s.nvals = 3;
  s.val_col[0] = qty;
  s.val_col[1] = price;
  s.val_col[2] = disc;
  s.val_type[0] = s.val_type[1] = s.val_type[2] = NUT_T_F64;
  s.naggs = 4;
  s.agg_op[0] = NUT_AGG_SUM;
  s.agg_expr[0] = NUT_EX_COL;
  s.agg_arg[0][0] = 0;
  s.agg_op[1] = NUT_AGG_SUM;
  s.agg_expr[1] = NUT_EX_COL;
  s.agg_arg[1][0] = 1;
  s.agg_op[2] = NUT_AGG_SUM;
  s.agg_expr[2] = NUT_EX_MUL_1M;
  s.agg_arg[2][0] = 1;
  s.agg_arg[2][1] = 2;
  s.agg_op[3] = NUT_AGG_COUNT;
  return nut_groupby(c, &s, 8, out);
}

}  // extern "C"
