// heavy.hpp — heavy keys split off before the ordered group-by's partition levels
// (aggregate.hip groupby_ordered).
//
// The range partition gives every key one level-1 partition, which holds ~1/16384 of the
// rows; a key with more rows than that (Zipf-like data: the top ~1000 keys of a 1e7-key pool
// hold ~45 % of the rows) would push its excess through the overflow arenas and aggregate
// on one workgroup.  Keys the host's sample saw often are instead aggregated here, in one
// streaming pass over the input: a host-built cuckoo table in LDS names them (two reads per
// lookup), their rows fold into LDS accumulators (merged into device words once per
// workgroup), and every other row is copied, compacted, to the arrays the partition levels
// then read.  scripts/tune/hk_tune.hip times it against a copy of the same arrays.
#pragma once

#include "agg_ops.hpp"
#include "common.hpp"
#include "gtable.hpp"

namespace nut {

constexpr int HK_THREADS = 256, HK_ITEMS = 8;
constexpr uint32_t HK_TILE = HK_THREADS * HK_ITEMS;  // rows per tile
constexpr int HK_MAX = 2048;                         // heavy keys at most
constexpr int HK_SLOTS = 8192;                       // cuckoo slots (load <= 1/4), host-built
constexpr int HK_WORDS = 2048;                       // heavy keys x aggregates at most (16 KB)

struct HkArgs {
  const uint64_t *key;
  const uint64_t *val[NUT_MAX_VALS];
  uint64_t *okey;                     // compacted rows (every row whose key is not heavy)
  uint64_t *oval[NUT_MAX_VALS];
  uint64_t n;
  uint64_t chunk;                     // tiles per workgroup: workgroup b reads tiles [b chunk, (b + 1) chunk)
  int nv, na;
  int32_t kind[NUT_MAX_AGGS];         // aggregate kinds (AggKind)
  int32_t arg[NUT_MAX_AGGS];          // value array of each aggregate (COUNT: unused)
  const int64_t *hk;                  // the heavy keys (h of them)
  const uint16_t *slot;               // [HK_SLOTS] cuckoo table: key index + 1 (0: empty), hk_slot1 / hk_slot2
  uint64_t seed1, seed2;
  uint32_t h;
  uint64_t *hagg;                     // [h x na] table-encoded words, initialised to agg_init
  uint64_t *count;                    // [gridDim.x] rows each workgroup kept
};

// a key's two cuckoo slots (the host places every heavy key in one of them: hk_cuckoo)
__host__ __device__ __forceinline__ uint32_t hk_slot(uint64_t k, uint64_t seed) {
  return (uint32_t)(mix64(k ^ seed) >> 32) & (HK_SLOTS - 1);
}

// host: a cuckoo table of the h keys (slot = key index + 1); false if some key found no
// place (the caller retries with other seeds)
inline bool hk_cuckoo(const int64_t *hk, uint32_t h, uint64_t s1, uint64_t s2, uint16_t *slot) {
  for (int i = 0; i < HK_SLOTS; ++i) slot[i] = 0;
  for (uint32_t j = 0; j < h; ++j) {
    uint16_t cur = (uint16_t)(j + 1);
    uint32_t pos = hk_slot((uint64_t)hk[j], s1);
    int steps = 0;
    for (;;) {
      const uint16_t old = slot[pos];
      slot[pos] = cur;
      if (!old) break;
      if (++steps > 1000) return false;
      cur = old;  // the evicted key moves to its other slot
      const uint64_t k = (uint64_t)hk[old - 1];
      const uint32_t a = hk_slot(k, s1), b = hk_slot(k, s2);
      pos = pos == a ? b : a;
    }
  }
  return true;
}

// a raw buffer resource over `bytes` bytes from p (stride 0; stores past `bytes` are
// discarded by the bounds check — how a dropped row's store writes nothing)
typedef unsigned int hk_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hk_rsrc(void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void hk_store(uint64_t v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  const hk_u32x2 w = {(uint32_t)v, (uint32_t)(v >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, (int)off, 0, 2);  // (glc 0, slc 1: non-temporal)
}

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

// Workgroup b owns a contiguous chunk of tiles and compacts its kept rows to the start of
// the same chunk of the output (no global cursor: the host reads the per-workgroup counts
// and hands the level-0 scatter one segment per workgroup).  Within a tile the kept rows of
// (item, wave) pairs get consecutive runs; the next tile's rows are loaded before this
// tile's are looked up.  NV: value arrays (registers for two tiles of them: a template, so
// one value array takes ~80 VGPRs, not the 206 that four would).  VAR: tuning variants for
// scripts/tune/hk_tune.hip (bit 0 no lookups, bit 1 no accumulator atomics, bit 2 no
// stores); the product runs VAR = 0.
template <int NV, int VAR = 0>
__global__ __launch_bounds__(HK_THREADS) void hk_split_kernel(HkArgs a) {
  __shared__ uint16_t s_slot[HK_SLOTS];  // cuckoo table: heavy key index + 1 (0: empty)
  __shared__ uint64_t s_key[HK_MAX];
  __shared__ uint64_t s_acc[HK_WORDS];
  __shared__ uint32_t s_off[2][HK_ITEMS * (HK_THREADS / 64)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = HK_THREADS / 64;
  for (int i = tid; i < HK_SLOTS; i += HK_THREADS) s_slot[i] = a.slot[i];
  for (uint32_t i = tid; i < a.h; i += HK_THREADS) s_key[i] = (uint64_t)a.hk[i];
  for (uint32_t i = tid; i < a.h * (uint32_t)a.na; i += HK_THREADS) s_acc[i] = agg_init(a.kind[i % a.na]);
  __syncthreads();
  const uint64_t ntiles = (a.n + HK_TILE - 1) / HK_TILE;
  const uint64_t t0 = (uint64_t)blockIdx.x * a.chunk, t1 = min(ntiles, t0 + a.chunk);
  uint64_t out = 0;  // this workgroup's next kept row, from its chunk's start
  // the chunk's output rows as buffer resources (< 2^32 bytes: the host checks)
  const uint32_t cbytes = (uint32_t)(a.chunk * HK_TILE * 8);
  const __amdgpu_buffer_rsrc_t rk = hk_rsrc(a.okey + t0 * HK_TILE, cbytes);
  __amdgpu_buffer_rsrc_t rv[NV > 0 ? NV : 1];
#pragma unroll
  for (int c = 0; c < NV; ++c) rv[c] = hk_rsrc(a.oval[c] + t0 * HK_TILE, cbytes);
  uint64_t k[HK_ITEMS], v[HK_ITEMS][NV];
  auto load = [&](uint64_t t) {
#pragma unroll
    for (int i = 0; i < HK_ITEMS; ++i) {
      const uint64_t r = min(t * HK_TILE + (uint64_t)i * HK_THREADS + tid, a.n - 1);  // (clamped: unconditional loads)
      k[i] = __builtin_nontemporal_load(a.key + r);
#pragma unroll
      for (int c = 0; c < NV; ++c) v[i][c] = __builtin_nontemporal_load(a.val[c] + r);
    }
  };
  if (t0 < t1) load(t0);
  int buf = 0;
  for (uint64_t t = t0; t < t1; ++t) {
    uint64_t ck[HK_ITEMS], cv[HK_ITEMS][NV];
#pragma unroll
    for (int i = 0; i < HK_ITEMS; ++i) {
      ck[i] = k[i];
#pragma unroll
      for (int c = 0; c < NV; ++c) cv[i][c] = v[i][c];
    }
    if (t + 1 < t1) load(t + 1);
    // lookups: a key's two cuckoo slots, then the keys they name — two rounds of 16 LDS
    // reads for all 8 rows of a lane, no probe loop
    int hid[HK_ITEMS];
    uint32_t j1[HK_ITEMS], j2[HK_ITEMS];
#pragma unroll
    for (int i = 0; i < HK_ITEMS; ++i) {
      j1[i] = (VAR & 1) ? 0u : s_slot[hk_slot(ck[i], a.seed1)];
      j2[i] = (VAR & 1) ? 0u : s_slot[hk_slot(ck[i], a.seed2)];
    }
#pragma unroll
    for (int i = 0; i < HK_ITEMS; ++i) {
      const uint64_t k1 = s_key[j1[i] ? j1[i] - 1 : 0], k2 = s_key[j2[i] ? j2[i] - 1 : 0];
      const bool in = t * HK_TILE + (uint64_t)i * HK_THREADS + tid < a.n;
      hid[i] = !in ? -2 : (j1[i] && k1 == ck[i]) ? (int)j1[i] - 1 : (j2[i] && k2 == ck[i]) ? (int)j2[i] - 1 : -1;
    }
    // the heavy rows into the accumulators: aggregate by aggregate (one kind dispatch per
    // aggregate and tile), every item inside
    for (int g = 0; g < a.na; ++g) {
      const int ag = a.arg[g];
      with_kind(a.kind[g], [&](auto KC) {
        constexpr int K = decltype(KC)::value;
#pragma unroll
        for (int i = 0; i < HK_ITEMS; ++i) {
          uint64_t x = 0;
#pragma unroll
          for (int c = 0; c < NV; ++c) x = ag == c ? cv[i][c] : x;
          if (!(VAR & 2) && hid[i] >= 0) fold_atomic<K>(&s_acc[hid[i] * a.na + g], x);
        }
      });
    }
    // compaction: the kept rows of item i, wave w go to one run; every lane stores (a fixed
    // number of stores per tile, so the next tile's loads are waited for by count, not by
    // vmcnt(0) behind this tile's stores), a dropped row (heavy, or past the end) at an
    // offset past the buffer, so its store writes nothing
    uint64_t m[HK_ITEMS];
#pragma unroll
    for (int i = 0; i < HK_ITEMS; ++i) {
      m[i] = __ballot(hid[i] == -1);
      if (lane == 0) s_off[buf][i * NW + wave] = (uint32_t)__popcll(m[i]);
    }
    __syncthreads();
    uint32_t before[HK_ITEMS], total = 0;
#pragma unroll
    for (int j = 0; j < HK_ITEMS * NW; ++j) {
      const uint32_t cj = s_off[buf][j];
      if (j % NW == wave) before[j / NW] = total;
      total += cj;
    }
#pragma unroll
    for (int i = 0; i < HK_ITEMS && !(VAR & 4); ++i) {
      const uint32_t o = hid[i] == -1 ? (uint32_t)(out + before[i] + lane_rank(m[i])) * 8u : 0xFFFFFFF0u;
      hk_store(ck[i], rk, o);
#pragma unroll
      for (int c = 0; c < NV; ++c) hk_store(cv[i][c], rv[c], o);
    }
    out += total;
    buf ^= 1;  // (the other half of s_off: the next tile's counts cannot overwrite these before every wave read them)
  }
  if (tid == 0) a.count[blockIdx.x] = out;
  __syncthreads();
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
