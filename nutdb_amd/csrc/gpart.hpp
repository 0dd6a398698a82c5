// gpart.hpp — partitioned aggregation for more groups than the on-chip tables hold
// (BASELINE config 3 at G = 1e5 .. 1e7).
//
// The streaming kernel (agg_kernel.hpp) first runs in SPILL mode: it evaluates WHERE and
// the aggregate arguments as always, but appends every passing row to staged arrays
// {k1, [k2], value arrays} instead of hashing it into a table (and counts the first
// partition level's histogram on the way).  The kernels here then
// radix-partition those records by the key hash (one or two 8-bit levels -> 256 or 65536
// partitions of a few hundred groups each), and the streaming kernel runs again in
// SEGMENT mode, one workgroup per partition: every group of a partition lives in that
// workgroup's LDS table, and the block-end merge into the global table inserts each group
// once, with no contention (partitions hold disjoint keys).
#pragma once

#include "common.hpp"

namespace nut {

constexpr int GP_THREADS = 512;
constexpr int GP_ITEMS = 16;
constexpr uint32_t GP_TILE = GP_THREADS * GP_ITEMS;  // 8192 records per scatter tile
constexpr int GP_HTHREADS = 256;
constexpr uint32_t GP_HTILE = 1u << 16;              // records per histogram tile
constexpr int GP_BINS = 256;
constexpr int GP_MAX_ARR = 3 + NUT_MAX_VALS;         // hash, k1, k2, value arrays

struct GpSeg {  // records [start, start + count) of the current buffer
  uint64_t start, count;
  uint32_t tile0, pad;  // first tile of the segment in the launch's tile table
};

struct GpArrays {
  const uint64_t *src[GP_MAX_ARR];  // [0] unused, [1] k1, [2] k2 (two keys), values
  uint64_t *dst[GP_MAX_ARR];
  int narr;
};

// the partition digit: a byte of the key tuple's owner hash (recomputed, never stored);
// kx (0 for the aggregation) re-keys the hash: the join table's home hash is
// owner_hash(k ^ kx) with its own kx, independent of the multi-GPU owner (kx = 0)
__device__ __forceinline__ uint32_t gp_digit(const uint64_t *k1, const uint64_t *k2, uint64_t i, int shift,
                                             uint64_t kx) {
  return (uint32_t)(owner_hash(k1[i] ^ kx, k2 ? k2[i] : 0, k2 ? 2 : 1) >> shift) & 255u;
}

// 256-bin histogram of (hash >> shift) & 255 per segment (gather: one for all segments)
__global__ __launch_bounds__(GP_HTHREADS) void gp_hist_kernel(const uint64_t *__restrict__ k1,
                                                              const uint64_t *__restrict__ k2,
                                                              const GpSeg *__restrict__ segs,
                                                              const uint32_t *__restrict__ tile_seg, int shift,
                                                              int gather, unsigned long long *__restrict__ hist,
                                                              uint64_t kx) {
  __shared__ uint32_t cnt[GP_BINS];
  const int tid = threadIdx.x;
  cnt[tid] = 0;
  __syncthreads();
  const uint32_t s = tile_seg[blockIdx.x];
  const GpSeg sg = segs[s];
  const uint64_t lo = sg.start + (uint64_t)(blockIdx.x - sg.tile0) * GP_HTILE;
  const uint32_t n = (uint32_t)min<uint64_t>(GP_HTILE, sg.start + sg.count - lo);
  for (uint32_t i = tid; i < n; i += GP_HTHREADS * 4) {
    uint32_t d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t k = i + j * GP_HTHREADS;
      d[j] = k < n ? gp_digit(k1, k2, lo + k, shift, kx) : 0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (i + j * GP_HTHREADS < n) atomicAdd(&cnt[d[j]], 1u);
  }
  __syncthreads();
  if (cnt[tid]) atomicAdd(&hist[(gather ? 0 : (uint64_t)s) * GP_BINS + tid], (unsigned long long)cnt[tid]);
}

// Unstable partition of every segment's records by (hash >> shift) & 255: a tile ranks its
// records with LDS atomics and claims each digit's output run with one global atomic on
// the segment's digit cursor; then every array is staged in LDS in digit order (one LDS
// write per record) and written out in coalesced runs.  Persistent (2 workgroups per CU):
// the keys stay in registers from the digit to their own staging, and the next tile's
// keys are fetched while this tile's value arrays go through.
// Gather mode: all segments share one set of 256 cursors (the spilled blocks' regions ->
// one compact partitioned array).
template <int NK, int T>
__global__ __launch_bounds__(T) void gp_scatter_kernel(GpArrays ar, const GpSeg *__restrict__ segs,
                                                                const uint32_t *__restrict__ tile_seg, uint32_t ntiles,
                                                                int shift, int gather,
                                                                unsigned long long *__restrict__ cursor, uint64_t kx) {
  __shared__ uint64_t s_stage[(T * GP_ITEMS)];
  __shared__ uint8_t s_dig[(T * GP_ITEMS)];
  __shared__ uint32_t s_cnt[GP_BINS];
  __shared__ uint32_t s_tex[GP_BINS];
  __shared__ uint64_t s_gb[GP_BINS];
  __shared__ uint32_t s_wsum[GP_BINS / kWave];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint64_t k1[GP_ITEMS], k2[NK == 2 ? GP_ITEMS : 1];
  auto load_keys = [&](uint32_t tt) {
    const GpSeg g = segs[tile_seg[tt]];
    const uint64_t lo = g.start + (uint64_t)(tt - g.tile0) * (T * GP_ITEMS);
    const uint32_t n = (uint32_t)min<uint64_t>((T * GP_ITEMS), g.start + g.count - lo);
#pragma unroll
    for (int i = 0; i < GP_ITEMS; ++i) {  // unconditional (clamped): all loads in flight at once
      const uint64_t r = lo + min((uint32_t)i * T + tid, n - 1);
      k1[i] = __builtin_nontemporal_load(ar.src[1] + r);
      if (NK == 2) k2[i] = __builtin_nontemporal_load(ar.src[2] + r);
    }
  };
  uint32_t t = blockIdx.x;
  if (t >= ntiles) return;
  load_keys(t);
  for (;;) {
    const uint32_t s = tile_seg[t];
    const GpSeg sg = segs[s];
    const uint64_t lo = sg.start + (uint64_t)(t - sg.tile0) * (T * GP_ITEMS);
    const uint32_t n = (uint32_t)min<uint64_t>((T * GP_ITEMS), sg.start + sg.count - lo);
    if (tid < GP_BINS) s_cnt[tid] = 0;
    __syncthreads();
    uint32_t dg[GP_ITEMS], slot[GP_ITEMS];
#pragma unroll
    for (int i = 0; i < GP_ITEMS; ++i) {
      const bool v = (uint32_t)i * T + tid < n;
      dg[i] = (uint32_t)(owner_hash(k1[i] ^ kx, NK == 2 ? k2[i] : 0, NK) >> shift) & 255u;
      slot[i] = v ? atomicAdd(&s_cnt[dg[i]], 1u) : 0u;
    }
    __syncthreads();
    uint32_t c = 0, incl = 0;
    if (tid < GP_BINS) {
      c = s_cnt[tid];
      incl = c;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
      }
      if (lane == 63) s_wsum[wave] = incl;
    }
    __syncthreads();
    if (tid < GP_BINS) {
      uint32_t add = 0;
#pragma unroll
      for (int w = 0; w < GP_BINS / kWave; ++w) add += (w < wave) ? s_wsum[w] : 0u;
      const uint32_t tex = incl - c + add;
      s_tex[tid] = tex;
      const uint64_t cs = gather ? 0 : (uint64_t)s;
      const uint64_t gb = c ? (uint64_t)atomicAdd(&cursor[cs * GP_BINS + tid], (unsigned long long)c) : 0;
      s_gb[tid] = gb - tex;  // output position of tile slot j with digit d = s_gb[d] + j
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < GP_ITEMS; ++i) {
      if ((uint32_t)i * T + tid < n) {
        slot[i] += s_tex[dg[i]];
        s_dig[slot[i]] = (uint8_t)dg[i];
      }
    }
    // one array through LDS: stage in digit order, write out coalesced runs
    auto pass = [&](const uint64_t (&v)[GP_ITEMS], uint64_t *dst) {
      __syncthreads();  // the previous array's write-out is done with s_stage
#pragma unroll
      for (int i = 0; i < GP_ITEMS; ++i)
        if ((uint32_t)i * T + tid < n) s_stage[slot[i]] = v[i];
      __syncthreads();
#pragma unroll
      for (int i = 0; i < GP_ITEMS; ++i) {
        const uint32_t j = (uint32_t)i * T + tid;
        if (j < n) dst[s_gb[s_dig[j]] + j] = s_stage[j];
      }
    };
    pass(k1, ar.dst[1]);
    if constexpr (NK == 2) pass(k2, ar.dst[2]);
    const uint32_t next = t + gridDim.x;
    if (next < ntiles) load_keys(next);  // the key registers are free
    for (int a = 3; a < ar.narr; ++a) {
      uint64_t v[GP_ITEMS];
#pragma unroll
      for (int i = 0; i < GP_ITEMS; ++i)
        v[i] = __builtin_nontemporal_load(ar.src[a] + lo + min((uint32_t)i * T + tid, n - 1));
      pass(v, ar.dst[a]);
    }
    if (next >= ntiles) break;
    __syncthreads();  // s_cnt / s_stage / s_dig / s_gb are reused
    t = next;
  }
}

}  // namespace nut
