// gtable.hpp — the global (HBM) group table shared by every group-by kernel:
// aggregate-word semantics, the find-or-claim protocol and the table maintenance
// kernels (init / compact / owner partition / rehash).
//
//   * single-key tables: the slot word IS the key (exact); the one key equal to the
//     empty marker lives in a dedicated extra slot (index cap);
//   * two-key tables: the key tuple is written to an arena entry FIRST and the slot word
//     {tag:32 | arena index:32} is published by the claiming CAS, so a reader never
//     waits for a half-written key;
//   * every cross-workgroup read of table words is a returning atomic (memory side),
//     never a plain or sc1 load that a stale line in this XCD's L2 could serve.
#pragma once

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
  uint32_t *ctl;     // [0] claimed, [1] flags (1 overflow), [2] special used, [3] arena used
                     //   ([0] and [3] are written by gtable_sum_kernel from the shards)
  uint32_t *shard;   // claim counters at [i * 16], arena counters at [(nsh + i) * 16]: one
                     //   64-B line each, so that inserts do not all hit one address
  int nsh_log2;      // 0 for small tables
  uint32_t limit_sh; // claims per shard before overflow is flagged
  uint32_t arena_sh; // arena entries per shard
  uint64_t cap;      // power of two
  uint32_t limit;    // claims allowed before overflow is flagged
  uint32_t arena_cap;
  int log2cap;
  int naggs;
  uint32_t kinds;    // 4 bits per aggregate kind
};

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
        if (atomicAdd(&t.shard[(s & ((1u << t.nsh_log2) - 1)) * 16], 1u) >= t.limit_sh) atomicOr(&t.ctl[1], 1u);
        return (int64_t)s;
      }
      if (old == h) return (int64_t)s;
    } else {
      uint64_t cur = rmw_load(&t.slot[s]);
      if (cur == kEmpty2) {
        if (word == kEmpty2) {
          const uint32_t sh = tag & ((1u << t.nsh_log2) - 1);
          const uint32_t loc = atomicAdd(&t.shard[((1u << t.nsh_log2) + sh) * 16], 1u);
          if (loc >= t.arena_sh) {
            atomicOr(&t.ctl[1], 1u);
            return -1;
          }
          const uint32_t idx = sh * t.arena_sh + loc;
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
          if (atomicAdd(&t.shard[(s & ((1u << t.nsh_log2) - 1)) * 16], 1u) >= t.limit_sh) atomicOr(&t.ctl[1], 1u);
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

// ctl[0] = claimed groups, ctl[3] = arena entries used (sums of the shard counters)
__global__ void gtable_sum_kernel(const GTable *__restrict__ gtp) {
  const GTable t = *gtp;
  const uint32_t nsh = 1u << t.nsh_log2;
  uint32_t c = 0, a = 0;
  for (uint32_t i = threadIdx.x; i < nsh; i += blockDim.x) {
    c += t.shard[i * 16];
    a += t.shard[(nsh + i) * 16];
  }
  __shared__ uint32_t sc[256], sa[256];
  sc[threadIdx.x] = c;
  sa[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tc = 0, ta = 0;
    for (uint32_t i = 0; i < blockDim.x; ++i) tc += sc[i], ta += sa[i];
    t.ctl[0] = tc;
    t.ctl[3] = ta;
  }
}

// dense column-major copy of the occupied slots; owner partitioning optional.  A block
// takes GT_CHUNK consecutive slots at a time, counts them per part in LDS (wave-aggregated
// when unpartitioned) and claims each part's run with ONE global atomic per chunk: a
// cursor atomic per wave serialised 10^7 groups on one address (6.3 ms).
constexpr int GT_THREADS = 256;  // the launch's block size
constexpr int GT_PER = 8;
constexpr uint32_t GT_CHUNK = GT_THREADS * GT_PER;
__global__ __launch_bounds__(GT_THREADS) void gtable_compact_kernel(const GTable *__restrict__ gtp, int nk,
                                                                    uint64_t *__restrict__ out, uint64_t out_cap,
                                                                    unsigned long long *__restrict__ cursors,
                                                                    int nparts, const uint64_t *__restrict__ seg_base) {
  __shared__ uint32_t s_cnt[64];
  __shared__ unsigned long long s_base[64];
  const GTable t = *gtp;
  const uint64_t stride = t.cap + 1;
  const int tid = threadIdx.x, lane = tid & 63;
  for (uint64_t c0 = (uint64_t)blockIdx.x * GT_CHUNK; c0 < stride; c0 += (uint64_t)gridDim.x * GT_CHUNK) {
    if (tid < nparts) s_cnt[tid] = 0;
    __syncthreads();
    uint64_t k1[GT_PER], k2[GT_PER];
    uint32_t rank[GT_PER];
    int part[GT_PER];
    bool occ[GT_PER];
    // slot words first, all in flight (clamped, unconditional), then the tuple lookups
    uint64_t wd[GT_PER];
#pragma unroll
    for (int i = 0; i < GT_PER; ++i) {
      const uint64_t sl = c0 + (uint64_t)i * GT_THREADS + tid;
      wd[i] = t.slot[sl < stride ? sl : stride - 1];
    }
#pragma unroll
    for (int i = 0; i < GT_PER; ++i) {
      const uint64_t sl = c0 + (uint64_t)i * GT_THREADS + tid;
      if (nk == 1) {
        k1[i] = sl == t.cap ? kEmpty : wd[i];
        k2[i] = 0;
        occ[i] = sl < stride && (sl == t.cap ? t.ctl[2] != 0u : wd[i] != kEmpty);
      } else {
        occ[i] = sl < t.cap && wd[i] != kEmpty2;
        const uint32_t ai = occ[i] ? (uint32_t)wd[i] : 0u;  // unconditional: the loads overlap
        k1[i] = (uint64_t)t.ak1[ai];
        k2[i] = (uint64_t)t.ak2[ai];
      }
    }
#pragma unroll
    for (int i = 0; i < GT_PER; ++i) {
      part[i] = 0;
      rank[i] = 0;
      if (nparts > 1) {
        if (occ[i]) {
          part[i] = (int)(owner_hash(k1[i], k2[i], nk) % (uint64_t)nparts);
          rank[i] = atomicAdd(&s_cnt[part[i]], 1u);
        }
      } else {
        const uint64_t m = __ballot(occ[i]);
        if (m) {
          const int leader = __builtin_ctzll(m);
          uint32_t b = 0;
          if (lane == leader) b = atomicAdd(&s_cnt[0], (uint32_t)__popcll(m));
          rank[i] = __shfl(b, leader, 64) + lane_rank(m);
        }
      }
    }
    __syncthreads();
    if (tid < nparts) s_base[tid] = s_cnt[tid] ? atomicAdd(&cursors[tid], (unsigned long long)s_cnt[tid]) : 0ull;
    __syncthreads();
    const int w = nk + t.naggs;
#pragma unroll
    for (int i = 0; i < GT_PER; ++i) {
      if (!occ[i]) continue;
      const uint64_t sl = c0 + (uint64_t)i * GT_THREADS + tid;
      const int pt = part[i];
      const uint64_t pos = s_base[pt] + rank[i];
      // segment `pt` starts at word w*seg_base[pt]; each of its columns has seg_n rows
      const uint64_t seg_n = nparts > 1 ? seg_base[nparts + pt] : out_cap;
      uint64_t *seg = out + (nparts > 1 ? (uint64_t)w * seg_base[pt] : 0);
      seg[pos] = k1[i];
      if (nk == 2) seg[seg_n + pos] = k2[i];
      for (int a = 0; a < t.naggs; ++a) {
        uint64_t x = t.agg[a * stride + sl];
        const int kind = kind_at(t.kinds, a);
        if (kind == AK_MIN_F64 || kind == AK_MAX_F64) x = ord_to_f64(x);
        seg[(uint64_t)(nk + a) * seg_n + pos] = x;
      }
    }
    __syncthreads();  // s_cnt / s_base are reused
  }
}

// groups per owner part: LDS counts per block chunk, one global atomic per (chunk, part)
__global__ __launch_bounds__(GT_THREADS) void gtable_owner_count_kernel(const GTable *__restrict__ gtp, int nk,
                                                                        int nparts, unsigned long long *counts) {
  __shared__ uint32_t s_cnt[64];
  const GTable t = *gtp;
  const uint64_t stride = t.cap + 1;
  const int tid = threadIdx.x;
  for (uint64_t c0 = (uint64_t)blockIdx.x * GT_CHUNK; c0 < stride; c0 += (uint64_t)gridDim.x * GT_CHUNK) {
    if (tid < nparts) s_cnt[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < GT_PER; ++i) {
      const uint64_t sl = c0 + (uint64_t)i * GT_THREADS + tid;
      uint64_t k1, k2;
      if (sl < stride && slot_keys(t, nk, sl, k1, k2)) atomicAdd(&s_cnt[owner_hash(k1, k2, nk) % (uint64_t)nparts], 1u);
    }
    __syncthreads();
    if (tid < nparts && s_cnt[tid]) atomicAdd(&counts[tid], (unsigned long long)s_cnt[tid]);
    __syncthreads();
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
