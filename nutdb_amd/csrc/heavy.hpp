// heavy.hpp — heavy keys split off before the ordered group-by's partition levels
// (aggregate.hip groupby_ordered).
//
// The range partition gives every key one level-1 partition, which holds ~1/16384 of the
// rows; a key with more rows than that (Zipf-like data: the top ~1000 keys of a 1e7-key pool
// hold ~45 % of the rows) would push its excess through the overflow arenas and aggregate
// on one workgroup.  Keys the host's sample saw often are instead aggregated here, in one
// streaming pass over the input: an LDS hash set names them, their rows fold into LDS
// accumulators (merged into device words once per workgroup), and every other row is
// copied, compacted, to the arrays the partition levels then read.
#pragma once

#include "agg_ops.hpp"
#include "common.hpp"
#include "gtable.hpp"

namespace nut {

constexpr int HK_THREADS = 256, HK_ITEMS = 8;
constexpr uint32_t HK_TILE = HK_THREADS * HK_ITEMS;  // rows per tile (one cursor claim)
constexpr int HK_MAX = 1024;                         // heavy keys at most
constexpr int HK_SLOTS = 2048;                       // LDS hash set (load <= 1/2)
constexpr int HK_WORDS = 4096;                       // heavy keys x aggregates at most (32 KB)

struct HkArgs {
  const uint64_t *key;
  const uint64_t *val[NUT_MAX_VALS];
  uint64_t *okey;                     // compacted rows (every row whose key is not heavy)
  uint64_t *oval[NUT_MAX_VALS];
  uint64_t n;
  int nv, na;
  int32_t kind[NUT_MAX_AGGS];         // aggregate kinds (AggKind)
  int32_t arg[NUT_MAX_AGGS];          // value array of each aggregate (COUNT: unused)
  const int64_t *hk;                  // the heavy keys (h of them)
  uint32_t h;
  uint64_t *hagg;                     // [h x na] table-encoded words, initialised to agg_init
  unsigned long long *cursor;         // compacted rows so far (output order: tile claims)
};

__device__ __forceinline__ uint32_t hk_hash(uint64_t k) { return (uint32_t)(mix64(k) >> 40) & (HK_SLOTS - 1); }

// combine an accumulator word into a shared one (both table-encoded)
template <int K>
__device__ __forceinline__ void combine_atomic(uint64_t *w, uint64_t x) {
  if constexpr (K == AK_SUM_F64) unsafeAtomicAdd((double *)w, as_f64(x));
  else if constexpr (K == AK_SUM_I64 || K == AK_COUNT) atomicAdd((unsigned long long *)w, (unsigned long long)x);
  else if constexpr (K == AK_MIN_F64) atomicMin((unsigned long long *)w, (unsigned long long)x);
  else if constexpr (K == AK_MAX_F64) atomicMax((unsigned long long *)w, (unsigned long long)x);
  else if constexpr (K == AK_MIN_I64) atomicMin((long long *)w, (long long)x);
  else atomicMax((long long *)w, (long long)x);
}

// Persistent: each workgroup claims tiles of HK_TILE rows in turn (grid stride); per tile
// the kept rows of (item, wave) pairs get consecutive output runs from one cursor claim.
__global__ __launch_bounds__(HK_THREADS) void hk_split_kernel(HkArgs a) {
  __shared__ uint16_t s_slot[HK_SLOTS];  // heavy key index + 1 (0: empty)
  __shared__ int64_t s_key[HK_MAX];
  __shared__ uint64_t s_acc[HK_WORDS];
  __shared__ uint32_t s_off[HK_ITEMS * (HK_THREADS / 64)];
  __shared__ uint64_t s_base;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = HK_THREADS / 64;
  for (int i = tid; i < HK_SLOTS; i += HK_THREADS) s_slot[i] = 0;
  for (uint32_t i = tid; i < a.h * (uint32_t)a.na; i += HK_THREADS) s_acc[i] = agg_init(a.kind[i % a.na]);
  __syncthreads();
  if (tid == 0) {  // (h <= HK_MAX keys into 2048 slots: linear probing always finds room)
    for (uint32_t j = 0; j < a.h; ++j) {
      s_key[j] = a.hk[j];
      uint32_t q = hk_hash((uint64_t)a.hk[j]);
      while (s_slot[q]) q = (q + 1) & (HK_SLOTS - 1);
      s_slot[q] = (uint16_t)(j + 1);
    }
  }
  __syncthreads();
  const uint64_t ntiles = (a.n + HK_TILE - 1) / HK_TILE;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t base = t * HK_TILE;
    uint64_t k[HK_ITEMS], v[HK_ITEMS][NUT_MAX_VALS];
    int hid[HK_ITEMS];
#pragma unroll
    for (int i = 0; i < HK_ITEMS; ++i) {
      const uint64_t r = base + (uint64_t)i * HK_THREADS + tid;
      const bool ok = r < a.n;
      k[i] = ok ? __builtin_nontemporal_load(a.key + r) : 0;
#pragma unroll
      for (int c = 0; c < NUT_MAX_VALS; ++c) v[i][c] = ok && c < a.nv ? __builtin_nontemporal_load(a.val[c] + r) : 0;
      hid[i] = ok ? -1 : -2;  // -2: past the end
    }
    // heavy lookup + in-place aggregation
#pragma unroll
    for (int i = 0; i < HK_ITEMS; ++i) {
      if (hid[i] == -1) {
        uint32_t q = hk_hash(k[i]);
        for (;;) {
          const uint32_t j = s_slot[q];
          if (!j) break;
          if ((uint64_t)s_key[j - 1] == k[i]) {
            hid[i] = (int)j - 1;
            break;
          }
          q = (q + 1) & (HK_SLOTS - 1);
        }
      }
      if (hid[i] >= 0) {
        for (int g = 0; g < a.na; ++g) {
          uint64_t x = 0;
#pragma unroll
          for (int c = 0; c < NUT_MAX_VALS; ++c) x = a.arg[g] == c ? v[i][c] : x;
          with_kind(a.kind[g], [&](auto KC) {
            constexpr int K = decltype(KC)::value;
            fold_atomic<K>(&s_acc[hid[i] * a.na + g], x);
          });
        }
      }
    }
    // compaction: the kept rows of item i, wave w go to one run
    uint64_t m[HK_ITEMS];
#pragma unroll
    for (int i = 0; i < HK_ITEMS; ++i) {
      m[i] = __ballot(hid[i] == -1);
      if (lane == 0) s_off[i * NW + wave] = (uint32_t)__popcll(m[i]);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t run = 0;
      for (int j = 0; j < HK_ITEMS * NW; ++j) {
        const uint32_t c = s_off[j];
        s_off[j] = run;
        run += c;
      }
      s_base = run ? (uint64_t)atomicAdd(a.cursor, (unsigned long long)run) : 0;
    }
    __syncthreads();
    const uint64_t ob = s_base;
#pragma unroll
    for (int i = 0; i < HK_ITEMS; ++i) {
      if (hid[i] == -1) {
        const uint64_t o = ob + s_off[i * NW + wave] + lane_rank(m[i]);
        __builtin_nontemporal_store(k[i], a.okey + o);
#pragma unroll
        for (int c = 0; c < NUT_MAX_VALS; ++c)
          if (c < a.nv) __builtin_nontemporal_store(v[i][c], a.oval[c] + o);
      }
    }
    __syncthreads();  // (s_off / s_base are rewritten by the next tile)
  }
  // this workgroup's heavy accumulators into the device words
  for (uint32_t i = tid; i < a.h * (uint32_t)a.na; i += HK_THREADS) {
    const int g = (int)(i % a.na);
    with_kind(a.kind[g], [&](auto KC) {
      constexpr int K = decltype(KC)::value;
      if (s_acc[i] != agg_init(K)) combine_atomic<K>(&a.hagg[i], s_acc[i]);
    });
  }
}

}  // namespace nut
