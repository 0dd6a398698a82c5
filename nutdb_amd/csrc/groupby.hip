// groupby.hip — fused  WHERE -> GROUP BY -> SUM/COUNT/MIN/MAX  (BASELINE configs 3, 4)
//
// Design:
//   * one streaming pass over the columns, 16 B per lane per load (two rows), grid sized
//     to the chip (blocks/CU from the LDS footprint) with grid-stride tiles;
//   * every workgroup owns an open-addressing hash table in LDS: fingerprint words,
//     then one 64-bit aggregate word per aggregate (SoA, so slots spread over banks);
//     rows update it with LDS atomics (ds_add_f64 / ds_add_u64 / ds_min,max_[ui]64).
//     f64 MIN/MAX use the IEEE total order mapped to u64 so the integer min/max
//     atomics apply;
//   * a block stops admitting NEW keys to its LDS table at 3/4 load; rows of keys it
//     has not admitted go straight to the global table (correct for any G, fast while
//     the hot keys fit on chip);
//   * at the end each block merges its occupied slots into the global (HBM) table with
//     device-scope atomics; claims there are CAS on the fingerprint word, performed at
//     the memory side, so no cross-XCD staleness is possible;
//   * single-key tables use the key itself as fingerprint (exact); the one key equal to
//     the empty marker lives in a dedicated extra slot.  Two-key tables fingerprint the
//     tuple and verify it against stored key words (ready-flag protocol).
// Algorithmic bytes: 8 B per referenced column per row (16 B/row for config 3,
// 48 B/row for config 4).
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

__host__ __device__ inline uint64_t agg_init(int kind) {
  switch (kind) {
    case AK_MIN_F64: return ~0ull;
    case AK_MAX_F64: return 0ull;
    case AK_MIN_I64: return 0x7FFFFFFFFFFFFFFFull;
    case AK_MAX_I64: return 0x8000000000000000ull;
    default: return 0ull;
  }
}

struct GTable {
  uint64_t *fp;      // [cap + 1]   slot `cap` = the empty-marker key (single-key tables)
  int64_t *k1;       // [cap + 1]   two-key tables only
  int64_t *k2;       // [cap + 1]
  uint32_t *ready;   // [cap + 1]
  uint64_t *agg;     // [naggs][cap + 1]
  uint32_t *ctl;     // [0] claimed, [1] flags (1 overflow, 2 timeout), [2] special used
  uint64_t cap;      // power of two
  uint32_t limit;    // claims allowed before overflow is flagged
  int log2cap;
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
  int32_t kind[NUT_MAX_AGGS];
  int32_t expr[NUT_MAX_AGGS];
  int32_t arg[NUT_MAX_AGGS][3];
  uint32_t lds_cap;     // power of two, 0 = no LDS table
  uint32_t lds_limit;
  int32_t lds_log2;
  GTable gt;
};

constexpr uint32_t G_SPIN_LIMIT = 1u << 22;

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

// ---- atomic update of one aggregate word (LDS or global: generic address space)
__device__ __forceinline__ void agg_update_lds(uint64_t *w, int kind, uint64_t x) {
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

// ---- global table: find or claim the slot of (fp, k1, k2); -1 on overflow
template <int NK>
__device__ __forceinline__ int64_t g_find(const GTable t, uint64_t fp, int64_t k1, int64_t k2) {
  if (NK == 1 && fp == kEmpty) {
    atomicOr(&t.ctl[2], 1u);
    return (int64_t)t.cap;
  }
  uint64_t s = slot_of(fp, t.log2cap);
  for (uint64_t probe = 0; probe < t.cap; ++probe) {
    uint64_t old = atomicCAS((unsigned long long *)&t.fp[s], (unsigned long long)kEmpty,
                             (unsigned long long)fp);
    const bool won = old == kEmpty;
    // claim block strictly before the wait block: a waiter never spins ahead of a
    // claimer of the same wave (no intra-wave spin deadlock)
    if (won) {
      uint32_t c = atomicAdd(&t.ctl[0], 1u);
      if (c >= t.limit) atomicOr(&t.ctl[1], 1u);
      if (NK == 2) {
        atomicExch((unsigned long long *)&t.k1[s], (unsigned long long)k1);
        atomicExch((unsigned long long *)&t.k2[s], (unsigned long long)k2);
        __hip_atomic_exchange(&t.ready[s], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (won) return (int64_t)s;
    if (old == fp) {
      if (NK == 1) return (int64_t)s;
      uint32_t spins = 0;
      bool timeout = false;
      while (rmw_load(&t.ready[s]) == 0u) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > G_SPIN_LIMIT) {
          timeout = true;
          break;
        }
      }
      if (timeout) {
        atomicOr(&t.ctl[1], 2u);
        return -1;
      }
      int64_t a = (int64_t)rmw_load((uint64_t *)&t.k1[s]);
      int64_t b = (int64_t)rmw_load((uint64_t *)&t.k2[s]);
      if (a == k1 && b == k2) return (int64_t)s;
    }
    s = (s + 1) & (t.cap - 1);
  }
  atomicOr(&t.ctl[1], 1u);
  return -1;
}

// LDS table view (dynamic shared memory, carved in this order, 16-B aligned)
struct LTable {
  uint64_t *fp;     // [cap + 1]
  uint64_t *agg;    // [naggs][cap + 1]
  int64_t *k1;      // [cap + 1] (NK == 2)
  int64_t *k2;
  uint32_t *ready;
  uint32_t *ctl;    // [0] claimed, [1] special used
};

template <int NK>
__device__ __forceinline__ int32_t l_find(const LTable &t, uint32_t cap, uint32_t limit, int log2cap,
                                          uint64_t fp, int64_t k1, int64_t k2) {
  if (NK == 1 && fp == kEmpty) {
    t.ctl[1] = 1u;
    return (int32_t)cap;
  }
  uint32_t s = slot_of(fp, log2cap);
  for (uint32_t probe = 0; probe < cap; ++probe) {
    uint64_t cur = t.fp[s];
    bool won = false;
    if (cur == kEmpty) {
      if (*(volatile uint32_t *)&t.ctl[0] >= limit) return -1;  // table closed to new keys
      cur = atomicCAS((unsigned long long *)&t.fp[s], (unsigned long long)kEmpty,
                      (unsigned long long)fp);
      won = cur == kEmpty;
      if (won) {
        atomicAdd(&t.ctl[0], 1u);
        if (NK == 2) {
          t.k1[s] = k1;
          t.k2[s] = k2;
          __hip_atomic_store(&t.ready[s], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
    if (won) return (int32_t)s;
    if (cur == fp) {
      if (NK == 1) return (int32_t)s;
      uint32_t spins = 0;
      while (__hip_atomic_load(&t.ready[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 20)) return -1;  // never expected; the global table is exact too
      }
      if (t.k1[s] == k1 && t.k2[s] == k2) return (int32_t)s;
    }
    s = (s + 1) & (cap - 1);
  }
  return -1;
}

template <int NK>
__device__ __forceinline__ void process_row(const AggArgs &p, const LTable &lt, bool use_lds,
                                            int64_t k1, int64_t k2,
                                            const uint64_t (&v)[NUT_MAX_VALS]) {
  uint64_t fp = NK == 1 ? (uint64_t)k1 : fp2((uint64_t)k1, (uint64_t)k2);
  int32_t ls = use_lds ? l_find<NK>(lt, p.lds_cap, p.lds_limit, p.lds_log2, fp, k1, k2) : -1;
  // all loops over aggregates are unrolled with compile-time indices: a runtime index
  // into the kernel-argument struct would spill the whole struct to scratch
  if (ls >= 0) {
    const uint32_t stride = p.lds_cap + 1;
#pragma unroll
    for (int a = 0; a < NUT_MAX_AGGS; ++a)
      if (a < p.naggs)
        agg_update_lds(&lt.agg[a * stride + ls], p.kind[a], p.kind[a] == AK_COUNT ? 0 : agg_value(p, a, v));
  } else {
    int64_t gs = g_find<NK>(p.gt, fp, k1, k2);
    if (gs < 0) return;
    const uint64_t stride = p.gt.cap + 1;
#pragma unroll
    for (int a = 0; a < NUT_MAX_AGGS; ++a)
      if (a < p.naggs)
        agg_update_lds(&p.gt.agg[a * stride + gs], p.kind[a], p.kind[a] == AK_COUNT ? 0 : agg_value(p, a, v));
  }
}

template <int NK>
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

__device__ __forceinline__ u64x2 ld2(const void *col, uint64_t i) {
  return *reinterpret_cast<const u64x2 *>((const uint64_t *)col + i);
}
__device__ __forceinline__ u64x2 ld2_tail(const void *col, uint64_t i, uint64_t n) {
  const uint64_t *c = (const uint64_t *)col;
  u64x2 r;
  r.x = i < n ? c[i] : 0;
  r.y = i + 1 < n ? c[i + 1] : 0;
  return r;
}

// Each lane handles 2 consecutive rows per step (one 16-B load per column).
template <int NK, bool TAIL>
__device__ __forceinline__ void process_pair(const AggArgs &p, const LTable &lt, bool use_lds, uint64_t i) {
  u64x2 kv1, kv2 = {0, 0};
  u64x2 pv[NUT_MAX_PRED];
  u64x2 vv[NUT_MAX_VALS];
#pragma unroll
  for (int t = 0; t < NUT_MAX_PRED; ++t)
    if (t < p.npred) pv[t] = TAIL ? ld2_tail(p.pred_col[t], i, p.n) : ld2(p.pred_col[t], i);
  kv1 = TAIL ? ld2_tail(p.keys[0], i, p.n) : ld2(p.keys[0], i);
  if (NK == 2) kv2 = TAIL ? ld2_tail(p.keys[1], i, p.n) : ld2(p.keys[1], i);
#pragma unroll
  for (int c = 0; c < NUT_MAX_VALS; ++c)
    if (c < p.nvals) vv[c] = TAIL ? ld2_tail(p.val_col[c], i, p.n) : ld2(p.val_col[c], i);

#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint64_t pr[NUT_MAX_PRED], vr[NUT_MAX_VALS];
#pragma unroll
    for (int t = 0; t < NUT_MAX_PRED; ++t) pr[t] = t < p.npred ? (r ? pv[t].y : pv[t].x) : 0;
#pragma unroll
    for (int c = 0; c < NUT_MAX_VALS; ++c) vr[c] = c < p.nvals ? (r ? vv[c].y : vv[c].x) : 0;
    bool ok = row_pass<NK>(p, pr) && (!TAIL || i + r < p.n);
    if (ok)
      process_row<NK>(p, lt, use_lds, (int64_t)(r ? kv1.y : kv1.x), (int64_t)(r ? kv2.y : kv2.x), vr);
  }
}

template <int NK>
__global__ __launch_bounds__(512) void agg_kernel(AggArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const uint32_t cap = p.lds_cap;
  const bool use_lds = cap != 0;
  const uint32_t stride = cap + 1;
  LTable lt;
  lt.fp = smem;
  lt.agg = lt.fp + stride;
  uint64_t *end = lt.agg + (size_t)p.naggs * stride;
  lt.k1 = (int64_t *)end;
  lt.k2 = lt.k1 + (NK == 2 ? stride : 0);
  lt.ready = (uint32_t *)(lt.k2 + (NK == 2 ? stride : 0));
  lt.ctl = lt.ready + (NK == 2 ? stride : 0);

  if (use_lds) {
    for (uint32_t s = threadIdx.x; s < stride; s += blockDim.x) {
      lt.fp[s] = kEmpty;
#pragma unroll
      for (int a = 0; a < NUT_MAX_AGGS; ++a)
        if (a < p.naggs) lt.agg[a * stride + s] = agg_init(p.kind[a]);
      if (NK == 2) lt.ready[s] = 0;
    }
    if (threadIdx.x < 2) lt.ctl[threadIdx.x] = 0;
    __syncthreads();
  }

  // grid-stride over pairs of rows
  const uint64_t npairs = (p.n + 1) / 2;
  const uint64_t full_pairs = p.n / 2;
  const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // main loop, 2 pairs in flight per lane
  for (; q + gstride < full_pairs; q += 2 * gstride) {
    process_pair<NK, false>(p, lt, use_lds, 2 * q);
    process_pair<NK, false>(p, lt, use_lds, 2 * (q + gstride));
  }
  for (; q < npairs; q += gstride) {
    if (q < full_pairs) process_pair<NK, false>(p, lt, use_lds, 2 * q);
    else process_pair<NK, true>(p, lt, use_lds, 2 * q);
  }

  if (!use_lds) return;
  __syncthreads();
  // merge the block's table into the global table
  for (uint32_t s = threadIdx.x; s < stride; s += blockDim.x) {
    bool occ = s < cap ? lt.fp[s] != kEmpty : lt.ctl[1] != 0u;
    if (!occ) continue;
    uint64_t fp = s < cap ? lt.fp[s] : kEmpty;
    int64_t k1 = NK == 1 ? (int64_t)fp : lt.k1[s];
    int64_t k2 = NK == 1 ? 0 : lt.k2[s];
    int64_t gs = g_find<NK>(p.gt, fp, k1, k2);
    if (gs < 0) continue;
    const uint64_t gstr = p.gt.cap + 1;
#pragma unroll
    for (int a = 0; a < NUT_MAX_AGGS; ++a)
      if (a < p.naggs) agg_merge_word(&p.gt.agg[a * gstr + gs], p.kind[a], lt.agg[a * stride + s]);
  }
}

// ---- global table init / compaction / partition
__global__ void gtable_init_kernel(GTable t, int naggs, const int32_t kinds0, const int32_t kinds1,
                                   const int32_t kinds2, const int32_t kinds3, const int32_t kinds4,
                                   const int32_t kinds5, const int32_t kinds6, const int32_t kinds7,
                                   int nk) {
  const int32_t kinds[8] = {kinds0, kinds1, kinds2, kinds3, kinds4, kinds5, kinds6, kinds7};
  const uint64_t stride = t.cap + 1;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < stride;
       s += (uint64_t)gridDim.x * blockDim.x) {
    t.fp[s] = kEmpty;
    for (int a = 0; a < naggs; ++a) t.agg[a * stride + s] = agg_init(kinds[a]);
    if (nk == 2) t.ready[s] = 0;
  }
}

// dense column-major copy of the occupied slots; owner partitioning optional
__global__ void gtable_compact_kernel(GTable t, int nk, int naggs, const int32_t *__restrict__ kinds,
                                      uint64_t *__restrict__ out, uint64_t out_cap,
                                      unsigned long long *__restrict__ cursors, int nparts,
                                      const uint64_t *__restrict__ seg_base) {
  const uint64_t stride = t.cap + 1;
  const int w = nk + naggs;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < stride;
       s += (uint64_t)gridDim.x * blockDim.x) {
    bool occ = s < t.cap ? t.fp[s] != kEmpty : (nk == 1 && t.ctl[2] != 0u);
    if (!occ) continue;
    uint64_t k1 = nk == 1 ? (s < t.cap ? t.fp[s] : kEmpty) : (uint64_t)t.k1[s];
    uint64_t k2 = nk == 2 ? (uint64_t)t.k2[s] : 0;
    int part = nparts > 1 ? (int)(owner_hash(k1, k2, nk) % (uint64_t)nparts) : 0;
    uint64_t pos = atomicAdd(&cursors[part], 1ull);
    // segment `part` starts at word w*seg_base[part]; column j of it has seg_n rows
    uint64_t seg_n = nparts > 1 ? seg_base[nparts + part] : out_cap;
    uint64_t *seg = out + (nparts > 1 ? (uint64_t)w * seg_base[part] : 0);
    seg[pos] = k1;
    if (nk == 2) seg[seg_n + pos] = k2;
    for (int a = 0; a < naggs; ++a) {
      uint64_t x = t.agg[a * stride + s];
      if (kinds[a] == AK_MIN_F64 || kinds[a] == AK_MAX_F64) x = ord_to_f64(x);
      seg[(uint64_t)(nk + a) * seg_n + pos] = x;
    }
  }
}

__global__ void gtable_owner_count_kernel(GTable t, int nk, int nparts, unsigned long long *counts) {
  const uint64_t stride = t.cap + 1;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < stride;
       s += (uint64_t)gridDim.x * blockDim.x) {
    bool occ = s < t.cap ? t.fp[s] != kEmpty : (nk == 1 && t.ctl[2] != 0u);
    if (!occ) continue;
    uint64_t k1 = nk == 1 ? (s < t.cap ? t.fp[s] : kEmpty) : (uint64_t)t.k1[s];
    uint64_t k2 = nk == 2 ? (uint64_t)t.k2[s] : 0;
    atomicAdd(&counts[owner_hash(k1, k2, nk) % (uint64_t)nparts], 1ull);
  }
}

}  // namespace nut

// ============================================================== host side
using namespace nut;

struct nut_groups {
  nut_ctx *ctx = nullptr;
  int nk = 1, naggs = 0;
  int32_t kinds[NUT_MAX_AGGS] = {0};
  GTable gt{};
  void *mem = nullptr;       // table allocation
  size_t mem_bytes = 0;
  int32_t *dev_kinds = nullptr;  // lives inside mem
  unsigned long long *dev_cursors = nullptr;  // [64] inside mem
  uint64_t *dev_segbase = nullptr;            // [2*64] inside mem
};

namespace {

int ilog2(uint64_t v) {
  int r = 0;
  while ((1ull << r) < v) ++r;
  return r;
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
      if (s->pred_type[t] != NUT_T_I64 && s->pred_type[t] != NUT_T_F64) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad predicate type");
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

size_t lds_bytes(uint32_t cap, int nk, int naggs) {
  if (cap == 0) return 0;
  size_t stride = cap + 1;
  size_t b = stride * 8 * (1 + naggs);
  if (nk == 2) b += stride * 16 + stride * 4;
  b += 16;
  return (b + 15) & ~size_t(15);
}

// (re)allocate the global table for `cap` slots
nut_status alloc_table(nut_groups *g, uint64_t cap) {
  const uint64_t stride = cap + 1;
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  size_t o_fp = carve(stride * 8);
  size_t o_agg = carve(stride * 8 * (size_t)std::max(g->naggs, 1));
  size_t o_k1 = g->nk == 2 ? carve(stride * 8) : 0;
  size_t o_k2 = g->nk == 2 ? carve(stride * 8) : 0;
  size_t o_rd = g->nk == 2 ? carve(stride * 4) : 0;
  size_t o_ctl = carve(64);
  size_t o_kinds = carve(64);
  size_t o_cur = carve(64 * 8);
  size_t o_seg = carve(128 * 8);
  if (g->mem && g->mem_bytes >= off) {
    // reuse
  } else {
    if (g->mem) (void)hipFree(g->mem);
    g->mem = nullptr;
    NUT_HIP(hipMalloc(&g->mem, off));
    g->mem_bytes = off;
  }
  char *b = (char *)g->mem;
  g->gt.fp = (uint64_t *)(b + o_fp);
  g->gt.agg = (uint64_t *)(b + o_agg);
  g->gt.k1 = g->nk == 2 ? (int64_t *)(b + o_k1) : nullptr;
  g->gt.k2 = g->nk == 2 ? (int64_t *)(b + o_k2) : nullptr;
  g->gt.ready = g->nk == 2 ? (uint32_t *)(b + o_rd) : nullptr;
  g->gt.ctl = (uint32_t *)(b + o_ctl);
  g->dev_kinds = (int32_t *)(b + o_kinds);
  g->dev_cursors = (unsigned long long *)(b + o_cur);
  g->dev_segbase = (uint64_t *)(b + o_seg);
  g->gt.cap = cap;
  g->gt.log2cap = ilog2(cap);
  g->gt.limit = (uint32_t)std::min<uint64_t>(cap - cap / 4, 0xFFFFFFF0ull);
  hipStream_t st = g->ctx->stream;
  NUT_HIP(hipMemsetAsync(g->gt.ctl, 0, 64, st));
  NUT_HIP(hipMemcpyAsync(g->dev_kinds, g->kinds, sizeof(g->kinds), hipMemcpyHostToDevice, st));
  const int32_t *k = g->kinds;
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)g->ctx->num_cus * 8);
  hipLaunchKernelGGL(gtable_init_kernel, dim3((unsigned)blocks), dim3(256), 0, st, g->gt, g->naggs,
                     k[0], k[1], k[2], k[3], k[4], k[5], k[6], k[7], g->nk);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

nut_status read_ctl(nut_groups *g, uint32_t *ctl3) {
  nut_ctx *c = g->ctx;
  NUT_HIP(hipMemcpyAsync(c->host_pinned, g->gt.ctl, 16, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  memcpy(ctl3, c->host_pinned, 12);
  return NUT_OK;
}

// launch the streaming aggregation of spec's rows into g's table
nut_status launch_agg(nut_groups *g, const nut_agg_spec *s, uint64_t group_hint) {
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
  for (int i = 0; i < s->naggs; ++i) {
    a.kind[i] = g->kinds[i];
    a.expr[i] = s->agg_op[i] == NUT_AGG_COUNT ? NUT_EX_COL : s->agg_expr[i];
    for (int j = 0; j < 3; ++j) a.arg[i][j] = s->agg_op[i] == NUT_AGG_COUNT ? 0 : s->agg_arg[i][j];
  }
  // all columns must be 16-B aligned for the vector loads
  auto misaligned = [](const void *p) { return ((uintptr_t)p & 15) != 0; };
  bool bad = misaligned(a.keys[0]) || misaligned(a.keys[1]);
  for (int t = 0; t < a.npred; ++t) bad |= misaligned(a.pred_col[t]);
  for (int v = 0; v < a.nvals; ++v) bad |= misaligned(a.val_col[v]);
  if (bad) return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: columns must be 16-byte aligned");

  // on-chip table: 2x the expected groups, within an LDS budget that keeps >= 1 block/CU
  const size_t lds_max = 160 * 1024;
  uint64_t want = group_hint ? 2 * group_hint : 4096;
  uint32_t lcap = 64;
  while (lcap < want && lds_bytes(lcap * 2, g->nk, g->naggs) <= lds_max) lcap *= 2;
  if (group_hint > 8ull * lcap) lcap = 0;  // hot keys cannot fit on chip: go straight to HBM
  a.lds_cap = lcap;
  a.lds_limit = lcap - lcap / 4;
  a.lds_log2 = lcap ? ilog2(lcap) : 0;
  a.gt = g->gt;
  size_t lb = lds_bytes(lcap, g->nk, g->naggs);
  int threads = 512;
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
nut_status ensure_room(nut_groups *g, uint64_t extra);

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
    if (!st) st = launch_agg(g, s, group_hint);
    uint32_t ctl[3] = {0, 0, 0};
    if (!st) st = read_ctl(g, ctl);
    if (st) {
      nut_groups_free(g);
      return st;
    }
    if (ctl[1] & 2u) {
      nut_groups_free(g);
      return fail(NUT_ERR_TIMEOUT, "nut_groupby: key publication spin limit hit");
    }
    if (!(ctl[1] & 1u)) break;
    // more groups than the table admits: retry with a larger table
    if (cap >= (1ull << 36) || attempt > 12) {
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
  for (int a = 0; a < s->naggs; ++a) {
    int32_t k = kind_of(s, a);
    bool same = k == g->kinds[a] || (g->kinds[a] == AK_COUNT && k == AK_SUM_I64);
    if (!same) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_accumulate: aggregate kinds differ");
  }
  DeviceGuard dg(c->device);
  g->ctx = c;
  st = ensure_room(g, s->n);
  if (st) return st;
  // COUNT partials merge by integer addition: the kernel's COUNT kind would add 1
  nut_groups tmp = *g;
  for (int a = 0; a < s->naggs; ++a)
    if (g->kinds[a] == AK_COUNT) tmp.kinds[a] = AK_SUM_I64;
  st = launch_agg(&tmp, s, s->n);
  if (st) return st;
  uint32_t ctl[3];
  st = read_ctl(g, ctl);
  if (st) return st;
  if (ctl[1]) return fail(ctl[1] & 2u ? NUT_ERR_TIMEOUT : NUT_ERR_OOM, "nut_groupby_accumulate: table overflow");
  return NUT_OK;
}

nut_status nut_groups_size(nut_groups *g, uint64_t *n) {
  if (!g || !n) return fail(NUT_ERR_INVALID_ARG, "nut_groups_size: NULL argument");
  DeviceGuard dg(g->ctx->device);
  uint32_t ctl[3];
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
  if (n > cap) return fail(NUT_ERR_CAPACITY, "nut_groups_to_device: capacity " + std::to_string(cap) +
                                                 " < " + std::to_string(n) + " groups");
  if (n == 0) return NUT_OK;
  if (!out) return fail(NUT_ERR_INVALID_ARG, "nut_groups_to_device: NULL output");
  nut_ctx *c = g->ctx;
  DeviceGuard dg(c->device);
  NUT_HIP(hipMemsetAsync(g->dev_cursors, 0, 64 * 8, c->stream));
  uint64_t stride = g->gt.cap + 1;
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)c->num_cus * 8);
  hipLaunchKernelGGL(gtable_compact_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, g->gt, g->nk,
                     g->naggs, g->dev_kinds, out, n, g->dev_cursors, 1, (const uint64_t *)nullptr);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

nut_status nut_groups_partition(nut_groups *g, int nparts, uint64_t *out, uint64_t cap, uint64_t *counts) {
  if (!g || !counts || nparts < 1 || nparts > 64)
    return fail(NUT_ERR_INVALID_ARG, "nut_groups_partition: bad argument");
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
  hipLaunchKernelGGL(gtable_owner_count_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, g->gt, g->nk,
                     nparts, g->dev_cursors);
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
  hipLaunchKernelGGL(gtable_compact_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, g->gt, g->nk,
                     g->naggs, g->dev_kinds, out, run, g->dev_cursors, nparts,
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
  if (n > cap) return fail(NUT_ERR_CAPACITY, "nut_groups_to_host: capacity " + std::to_string(cap) +
                                                 " < " + std::to_string(n) + " groups");
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

nut_status nut_groupby_i64_f64(nut_ctx *c, const int64_t *key, const double *val, uint64_t n,
                               uint32_t mask, uint64_t group_hint, nut_groups **out) {
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
  s.agg_op[0] = NUT_AGG_SUM;  s.agg_expr[0] = NUT_EX_COL;    s.agg_arg[0][0] = 0;
  s.agg_op[1] = NUT_AGG_SUM;  s.agg_expr[1] = NUT_EX_COL;    s.agg_arg[1][0] = 1;
  s.agg_op[2] = NUT_AGG_SUM;  s.agg_expr[2] = NUT_EX_MUL_1M; s.agg_arg[2][0] = 1; s.agg_arg[2][1] = 2;
  s.agg_op[3] = NUT_AGG_COUNT;
  return nut_groupby(c, &s, 8, out);
}

}  // extern "C"

namespace {
__global__ void rehash_kernel(GTable src, GTable dst, int nk, int naggs, const int32_t *__restrict__ kinds) {
  const uint64_t stride = src.cap + 1;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < stride;
       s += (uint64_t)gridDim.x * blockDim.x) {
    bool occ = s < src.cap ? src.fp[s] != kEmpty : (nk == 1 && src.ctl[2] != 0u);
    if (!occ) continue;
    uint64_t fp = s < src.cap ? src.fp[s] : kEmpty;
    int64_t k1 = nk == 1 ? (int64_t)fp : src.k1[s];
    int64_t k2 = nk == 1 ? 0 : src.k2[s];
    int64_t d = nk == 1 ? g_find<1>(dst, fp, k1, k2) : g_find<2>(dst, fp, k1, k2);
    if (d < 0) continue;
    for (int a = 0; a < naggs; ++a)
      agg_merge_word(&dst.agg[a * (dst.cap + 1) + d], kinds[a], src.agg[a * stride + s]);
  }
}

nut_status ensure_room(nut_groups *g, uint64_t extra) {
  uint32_t ctl[3];
  nut_status st = read_ctl(g, ctl);
  if (st) return st;
  uint64_t need = (uint64_t)ctl[0] + extra + 1;
  if (need <= g->gt.limit) return NUT_OK;
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
  hipLaunchKernelGGL(rehash_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, g->gt, fresh.gt, g->nk,
                     g->naggs, fresh.dev_kinds);
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipStreamSynchronize(c->stream));
  (void)hipFree(g->mem);
  g->mem = fresh.mem;
  g->mem_bytes = fresh.mem_bytes;
  g->gt = fresh.gt;
  g->dev_kinds = fresh.dev_kinds;
  g->dev_cursors = fresh.dev_cursors;
  g->dev_segbase = fresh.dev_segbase;
  fresh.mem = nullptr;
  return NUT_OK;
}
}  // namespace
