// filter_tune.hip — standalone variant sweep for the filter/compaction kernel
// (not part of the product; build: hipcc --offload-arch=gfx950 -O3 -std=c++17
//  -I include scripts/tune/filter_tune.hip -o /tmp/filter_tune).
// Times each variant with hipEvents over R launches at N rows, s = 0.5, and checks the
// output count + checksum against variant 0.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../../nutdb_amd/csrc/common.hpp"

using namespace nut;

constexpr uint64_t FLAG_AGG = 1ull << 62;
constexpr uint64_t FLAG_INC = 2ull << 62;
constexpr uint64_t VAL_MASK = (1ull << 62) - 1;

template <int LB>
__device__ uint64_t lookback(uint64_t *__restrict__ status, uint32_t tile, uint64_t total, int lane, int sleep) {
  if (tile == 0) {
    if (lane == 0) st_agent(&status[0], FLAG_INC | total);
    return 0;
  }
  if (lane == 0) st_agent(&status[tile], FLAG_AGG | total);
  uint64_t excl = 0;
  int64_t pred = (int64_t)tile - 1;
  uint32_t spins = 0;
  for (;;) {
    uint64_t s[LB];
#pragma unroll
    for (int m = 0; m < LB; ++m) {
      int64_t idx = pred - m * 64 - lane;
      s[m] = idx >= 0 ? ld_agent(&status[idx]) : FLAG_INC;
    }
    bool done = false;
#pragma unroll
    for (int m = 0; m < LB; ++m) {
      int64_t idx = pred - m * 64 - lane;
      while (__any((s[m] >> 62) == 0)) {
        if (sleep) __builtin_amdgcn_s_sleep(1);
        if ((s[m] >> 62) == 0) s[m] = ld_agent(&status[idx]);
        if (++spins > (1u << 22)) s[m] = FLAG_INC | (s[m] & VAL_MASK);
      }
      uint64_t inc = __ballot((s[m] >> 62) == 2);
      if (inc) {
        int first = __builtin_ctzll(inc);
        excl += wave_sum_u64(lane <= first ? (s[m] & VAL_MASK) : 0);
        done = true;
        break;
      }
      excl += wave_sum_u64(s[m] & VAL_MASK);
    }
    if (done) break;
    pred -= 64 * LB;
  }
  if (lane == 0) st_agent(&status[tile], FLAG_INC | (excl + total));
  return excl;
}

// THREADS x (STRIPES x 2 rows) per tile.  LDS: stage the tile's selected values and
// write them out contiguously.  NT: non-temporal loads.
template <int THREADS, int STRIPES, bool LDS, bool NT, int SLEEP, bool TICKET = true, int LB = 1, int MODE = 0, bool NTS = false>
__global__ __launch_bounds__(THREADS) void filt(const int64_t *__restrict__ col, uint64_t n, int64_t k,
                                                int64_t *__restrict__ out, uint64_t *__restrict__ out_n,
                                                uint32_t *__restrict__ ticket, uint64_t *__restrict__ status,
                                                uint32_t ntiles) {
  constexpr int WAVES = THREADS / kWave;
  constexpr int SROWS = THREADS * 2;
  constexpr int TILE = SROWS * STRIPES;
  __shared__ uint32_t s_tile;
  __shared__ uint32_t s_cnt[STRIPES][WAVES];
  __shared__ uint64_t s_excl, s_total;
  __shared__ int64_t s_out[LDS ? TILE : 1];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (TICKET) {
    if (tid == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
  }
  const uint32_t tile = TICKET ? s_tile : blockIdx.x;
  const uint64_t base = (uint64_t)tile * TILE;
  const bool full = base + TILE <= n;
  int64_t v0[STRIPES], v1[STRIPES];
#pragma unroll
  for (int j = 0; j < STRIPES; ++j) {
    uint64_t idx = base + j * SROWS + 2 * tid;
    if (full) {
      i64x2 v;
      if (NT)
        v = __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(col + idx));
      else
        v = *reinterpret_cast<const i64x2 *>(col + idx);
      v0[j] = v.x;
      v1[j] = v.y;
    } else {
      v0[j] = idx < n ? col[idx] : 0;
      v1[j] = idx + 1 < n ? col[idx + 1] : 0;
    }
  }
  uint32_t r0[STRIPES];
  uint32_t sel = 0;
#pragma unroll
  for (int j = 0; j < STRIPES; ++j) {
    uint64_t idx = base + j * SROWS + 2 * tid;
    bool p0 = v0[j] < k && (full || idx < n);
    bool p1 = v1[j] < k && (full || idx + 1 < n);
    uint64_t b0 = __ballot(p0), b1 = __ballot(p1);
    r0[j] = lane_rank(b0) + lane_rank(b1);
    sel |= (p0 ? 1u : 0u) << (2 * j);
    sel |= (p1 ? 1u : 0u) << (2 * j + 1);
    if (lane == 0) s_cnt[j][wave] = (uint32_t)(__popcll(b0) + __popcll(b1));
  }
  __syncthreads();
  if (wave == 0) {
    uint32_t c = 0;
    for (int i = lane; i < STRIPES * WAVES; i += 64) c += (&s_cnt[0][0])[i];
    uint64_t total = wave_sum_u64(c);
    uint64_t excl = (MODE == 1 || MODE == 3) ? base : lookback<LB>(status, tile, total, lane, SLEEP);
    if (lane == 0) {
      s_excl = excl;
      s_total = total;
      if (tile == ntiles - 1) *out_n = excl + total;
    }
  }
  if (LDS) {
    uint32_t off = 0;
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) {
      uint32_t before = 0;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) before += (w < wave) ? s_cnt[j][w] : 0u;
      uint32_t pos = off + before + r0[j];
      bool p0 = (sel >> (2 * j)) & 1u, p1 = (sel >> (2 * j + 1)) & 1u;
      if (p0) s_out[pos] = v0[j];
      if (p1) s_out[pos + (p0 ? 1 : 0)] = v1[j];
#pragma unroll
      for (int w = 0; w < WAVES; ++w) off += s_cnt[j][w];
    }
    __syncthreads();
    const uint64_t o = s_excl;
    const uint32_t T = (uint32_t)s_total;
    if (MODE != 2)
      for (uint32_t i = tid; i < T; i += THREADS) out[o + i] = s_out[i];
  } else {
    __syncthreads();
    uint64_t off = s_excl;
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) {
      uint64_t before = 0;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) before += (w < wave) ? s_cnt[j][w] : 0u;
      uint64_t pos = off + before + r0[j];
      bool p0 = (sel >> (2 * j)) & 1u, p1 = (sel >> (2 * j + 1)) & 1u;
      if (MODE != 2 && MODE != 3) {
        if (NTS) {
          if (p0) __builtin_nontemporal_store(v0[j], &out[pos]);
          if (p1) __builtin_nontemporal_store(v1[j], &out[pos + (p0 ? 1 : 0)]);
        } else {
          if (p0) out[pos] = v0[j];
          if (p1) out[pos + (p0 ? 1 : 0)] = v1[j];
        }
      }
#pragma unroll
      for (int w = 0; w < WAVES; ++w) off += s_cnt[j][w];
    }
  }
}

__global__ void gen(int64_t *c, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c[i] = (int64_t)(gen_u64(0x2A, i) >> 2);
}

__global__ void copyk(const int64_t *__restrict__ a, int64_t *__restrict__ b, uint64_t n) {
  for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 2; i < n; i += (uint64_t)gridDim.x * blockDim.x * 2) {
    i64x2 v = *reinterpret_cast<const i64x2 *>(a + i);
    if ((i & 3) == 0) *reinterpret_cast<i64x2 *>(b + i / 2) = v;
  }
}

// better copy: 4 x 16 B loads in flight per thread, grid-stride
__global__ __launch_bounds__(256) void copy4(const int64_t *__restrict__ a, int64_t *__restrict__ b, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * 8;
  for (uint64_t i = blockIdx.x * 2048ull + threadIdx.x * 2; i < n; i += stride) {
    i64x2 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint64_t q = i + (uint64_t)j * 512;
      v[j] = q + 1 < n ? *reinterpret_cast<const i64x2 *>(a + q) : i64x2{0, 0};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint64_t q = i + (uint64_t)j * 512;
      if (q + 1 < n && (j & 1) == 0) *reinterpret_cast<i64x2 *>(b + q / 2) = v[j] + v[j + 1];
    }
  }
}

// read 8n, write 4n (every other 16-B vector): the HBM ceiling for a 2:1 read:write stream
template <int LOADS, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copyN(const int64_t *__restrict__ a, int64_t *__restrict__ b, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 512 * LOADS;
  for (uint64_t i = blockIdx.x * 512ull * LOADS + threadIdx.x * 2; i < n; i += stride) {
    i64x2 v[LOADS];
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      uint64_t q = i + (uint64_t)j * 512;
      if (NTL)
        v[j] = q + 1 < n ? __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(a + q)) : i64x2{0, 0};
      else
        v[j] = q + 1 < n ? *reinterpret_cast<const i64x2 *>(a + q) : i64x2{0, 0};
    }
#pragma unroll
    for (int j = 0; j < LOADS; j += 2) {
      uint64_t q = i + (uint64_t)j * 512;
      i64x2 w = v[j] + v[j + 1];
      i64x2 *d = reinterpret_cast<i64x2 *>(b + (q - threadIdx.x * 2) / 2 + threadIdx.x * 2);
      if (q + 1 < n) {
        if (NTS)
          __builtin_nontemporal_store(w, d);
        else
          *d = w;
      }
    }
  }
}

__global__ void checksum(const int64_t *o, uint64_t n, unsigned long long *h) {
  unsigned long long s = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    s += (unsigned long long)o[i] * (i + 1);
  atomicAdd(h, s);
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));            \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <int THREADS, int STRIPES, bool LDS, bool NT, int SLEEP, bool TICKET = true, int LB = 1, int MODE = 0, bool NTS = false>
void run(const char *name, const int64_t *col, uint64_t n, int64_t k, int64_t *out, uint64_t *dn, void *state,
         int R, unsigned long long *dh) {
  constexpr int TILE = THREADS * 2 * STRIPES;
  uint32_t ntiles = (uint32_t)((n + TILE - 1) / TILE);
  size_t sb = 16 + (size_t)ntiles * 8;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float tot = 0;
  for (int r = 0; r < R + 2; ++r) {
    CK(hipMemsetAsync(state, 0, sb, 0));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((filt<THREADS, STRIPES, LDS, NT, SLEEP, TICKET, LB, MODE, NTS>), dim3(ntiles), dim3(THREADS), 0, 0, col, n, k, out, dn,
                       (uint32_t *)state, (uint64_t *)((char *)state + 16), ntiles);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) tot += ms;
  }
  uint64_t cnt;
  CK(hipMemcpy(&cnt, dn, 8, hipMemcpyDeviceToHost));
  CK(hipMemset(dh, 0, 8));
  hipLaunchKernelGGL(checksum, dim3(1024), dim3(256), 0, 0, out, cnt, dh);
  unsigned long long h;
  CK(hipMemcpy(&h, dh, 8, hipMemcpyDeviceToHost));
  double ms = tot / R;
  double gb = (8.0 * n + 8.0 * cnt) / 1e9;
  printf("%-34s %8.4f ms  %7.1f GB/s  count=%llu hash=%016llx\n", name, ms, gb / (ms * 1e-3),
         (unsigned long long)cnt, h);
}


// persistent, software-pipelined: block b handles tiles b, b+G, ...; the next tile's
// loads are in flight while the current tile does its look-back and stores
template <int THREADS, int STRIPES, bool NT, int OCC>
__global__ __launch_bounds__(THREADS, OCC) void filt_p(const int64_t *__restrict__ col, uint64_t n, int64_t k,
                                                  int64_t *__restrict__ out, uint64_t *__restrict__ out_n,
                                                  uint64_t *__restrict__ status, uint32_t ntiles) {
  constexpr int WAVES = THREADS / kWave;
  constexpr int SROWS = THREADS * 2;
  constexpr int TILE = SROWS * STRIPES;
  __shared__ uint32_t s_cnt[STRIPES][WAVES];
  __shared__ uint64_t s_excl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t G = gridDim.x;
  i64x2 cur[STRIPES], nxt[STRIPES];
  auto load = [&](i64x2(&v)[STRIPES], uint32_t t) {
    const uint64_t base = (uint64_t)t * TILE;
    const bool full = base + TILE <= n;
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) {
      const uint64_t idx = base + j * SROWS + 2 * tid;
      if (full) {
        if (NT)
          v[j] = __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(col + idx));
        else
          v[j] = *reinterpret_cast<const i64x2 *>(col + idx);
      } else {
        v[j].x = idx < n ? col[idx] : 0;
        v[j].y = idx + 1 < n ? col[idx + 1] : 0;
      }
    }
  };
  uint32_t tile = blockIdx.x;
  if (tile < ntiles) load(cur, tile);
  for (; tile < ntiles; tile += G) {
    const uint32_t nt = tile + G;
    if (nt < ntiles) load(nxt, nt);
    const uint64_t base = (uint64_t)tile * TILE;
    const bool full = base + TILE <= n;
    uint32_t r0[STRIPES];
    uint32_t sel = 0;
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) {
      const uint64_t idx = base + j * SROWS + 2 * tid;
      bool p0 = cur[j].x < k && (full || idx < n);
      bool p1 = cur[j].y < k && (full || idx + 1 < n);
      uint64_t b0 = __ballot(p0), b1 = __ballot(p1);
      r0[j] = lane_rank(b0) + lane_rank(b1);
      sel |= (p0 ? 1u : 0u) << (2 * j);
      sel |= (p1 ? 1u : 0u) << (2 * j + 1);
      if (lane == 0) s_cnt[j][wave] = (uint32_t)(__popcll(b0) + __popcll(b1));
    }
    __syncthreads();
    if (wave == 0) {
      uint32_t c = 0;
      for (int i = lane; i < STRIPES * WAVES; i += 64) c += (&s_cnt[0][0])[i];
      uint64_t total = wave_sum_u64(c);
      uint64_t excl = lookback<1>(status, tile, total, lane, 1);
      if (lane == 0) {
        s_excl = excl;
        if (tile == ntiles - 1) *out_n = excl + total;
      }
    }
    __syncthreads();
    uint64_t off = s_excl;
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) {
      uint64_t before = 0;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) before += (w < wave) ? s_cnt[j][w] : 0u;
      uint64_t pos = off + before + r0[j];
      bool p0 = (sel >> (2 * j)) & 1u, p1 = (sel >> (2 * j + 1)) & 1u;
      if (p0) out[pos] = cur[j].x;
      if (p1) out[pos + (p0 ? 1 : 0)] = cur[j].y;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) off += s_cnt[j][w];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) cur[j] = nxt[j];
  }
}

template <int THREADS, int STRIPES, bool NT, int OCC>
void run_p(const char *name, const int64_t *col, uint64_t n, int64_t k, int64_t *out, uint64_t *dn, void *state,
           int R, unsigned long long *dh, int gridmul) {
  constexpr int TILE = THREADS * 2 * STRIPES;
  uint32_t ntiles = (uint32_t)((n + TILE - 1) / TILE);
  size_t sb = 16 + (size_t)ntiles * 8;
  int per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, filt_p<THREADS, STRIPES, NT, OCC>, THREADS, 0));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  uint32_t grid = (uint32_t)std::min<uint64_t>(ntiles, (uint64_t)per_cu * prop.multiProcessorCount * gridmul / 4);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float tot = 0;
  for (int r = 0; r < R + 2; ++r) {
    CK(hipMemsetAsync(state, 0, sb, 0));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((filt_p<THREADS, STRIPES, NT, OCC>), dim3(grid), dim3(THREADS), 0, 0, col, n, k, out, dn,
                       (uint64_t *)((char *)state + 16), ntiles);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) tot += ms;
  }
  uint64_t cnt;
  CK(hipMemcpy(&cnt, dn, 8, hipMemcpyDeviceToHost));
  CK(hipMemset(dh, 0, 8));
  hipLaunchKernelGGL(checksum, dim3(1024), dim3(256), 0, 0, out, cnt, dh);
  unsigned long long h;
  CK(hipMemcpy(&h, dh, 8, hipMemcpyDeviceToHost));
  double ms = tot / R;
  double gb = (8.0 * n + 8.0 * cnt) / 1e9;
  printf("%-28s occ%d g%-5u %8.4f ms  %7.1f GB/s  count=%llu hash=%016llx\n", name, per_cu, grid, ms,
         gb / (ms * 1e-3), (unsigned long long)cnt, h);
}

// dedicated look-back wave: THREADS data lanes + 1 wave that walks the predecessors'
// statuses while the data waves' loads are in flight (its vmcnt holds no data loads).
// The tile's AGG is published by the last data wave to finish counting (LDS counter),
// independent of the walk; the walker publishes INC.
template <int THREADS, int STRIPES, bool TICKET>
__global__ __launch_bounds__(THREADS + 64) void filt_w(const int64_t *__restrict__ col, uint64_t n, int64_t k,
                                                     int64_t *__restrict__ out, uint64_t *__restrict__ out_n,
                                                     uint32_t *__restrict__ ticket, uint64_t *__restrict__ status,
                                                     uint32_t ntiles) {
  constexpr int WAVES = THREADS / kWave;
  constexpr int SROWS = THREADS * 2;
  constexpr int TILE = SROWS * STRIPES;
  __shared__ uint32_t s_cnt[STRIPES][WAVES];
  __shared__ uint32_t s_total, s_done, s_tile;
  __shared__ uint64_t s_excl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    s_total = 0;
    s_done = 0;
    if (TICKET) s_tile = atomicAdd(ticket, 1u);
  }
  __syncthreads();
  const uint32_t tile = TICKET ? s_tile : blockIdx.x;
  if (wave == WAVES) {
    // ---- walker
    uint64_t excl = 0;
    if (tile > 0) {
      int64_t pred = (int64_t)tile - 1;
      uint32_t spins = 0;
      for (;;) {
        int64_t idx = pred - lane;
        uint64_t st = idx >= 0 ? ld_agent(&status[idx]) : FLAG_INC;
        while (__any((st >> 62) == 0)) {
          __builtin_amdgcn_s_sleep(1);
          if ((st >> 62) == 0) st = ld_agent(&status[idx]);
          if (++spins > (1u << 22)) st = FLAG_INC | (st & VAL_MASK);
        }
        uint64_t inc = __ballot((st >> 62) == 2);
        if (inc) {
          int first = __builtin_ctzll(inc);
          excl += wave_sum_u64(lane <= first ? (st & VAL_MASK) : 0);
          break;
        }
        excl += wave_sum_u64(st & VAL_MASK);
        pred -= kWave;
      }
    }
    // wait for the data waves' total (LDS), publish INC
    uint32_t done;
    do {
      done = __hip_atomic_load(&s_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    } while (done != WAVES);
    const uint64_t total = __hip_atomic_load(&s_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (lane == 0) {
      st_agent(&status[tile], FLAG_INC | (excl + total));
      s_excl = excl;
      if (tile == ntiles - 1) *out_n = excl + total;
    }
    __syncthreads();
    return;
  }
  // ---- data waves
  const uint64_t base = (uint64_t)tile * TILE;
  const bool full = base + TILE <= n;
  int64_t v0[STRIPES], v1[STRIPES];
#pragma unroll
  for (int j = 0; j < STRIPES; ++j) {
    uint64_t idx = base + j * SROWS + 2 * tid;
    if (full) {
      i64x2 v = *reinterpret_cast<const i64x2 *>(col + idx);
      v0[j] = v.x;
      v1[j] = v.y;
    } else {
      v0[j] = idx < n ? col[idx] : 0;
      v1[j] = idx + 1 < n ? col[idx + 1] : 0;
    }
  }
  uint32_t r0[STRIPES];
  uint32_t sel = 0, mine = 0;
#pragma unroll
  for (int j = 0; j < STRIPES; ++j) {
    uint64_t idx = base + j * SROWS + 2 * tid;
    bool p0 = v0[j] < k && (full || idx < n);
    bool p1 = v1[j] < k && (full || idx + 1 < n);
    uint64_t b0 = __ballot(p0), b1 = __ballot(p1);
    r0[j] = lane_rank(b0) + lane_rank(b1);
    sel |= (p0 ? 1u : 0u) << (2 * j);
    sel |= (p1 ? 1u : 0u) << (2 * j + 1);
    uint32_t c = (uint32_t)(__popcll(b0) + __popcll(b1));
    if (lane == 0) s_cnt[j][wave] = c;
    mine += c;
  }
  if (lane == 0) {
    uint32_t t = atomicAdd(&s_total, mine) + mine;
    uint32_t d = __hip_atomic_fetch_add(&s_done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) + 1;
    if (d == WAVES) {
      // last data wave: every wave's count is in s_total; publish AGG now
      uint32_t tot = __hip_atomic_load(&s_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (tile == 0)
        ;  // tile 0's walker publishes INC with excl = 0
      else
        st_agent(&status[tile], FLAG_AGG | tot);
    }
    (void)t;
  }
  __syncthreads();
  uint64_t off = s_excl;
#pragma unroll
  for (int j = 0; j < STRIPES; ++j) {
    uint64_t before = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) before += (w < wave) ? s_cnt[j][w] : 0u;
    uint64_t pos = off + before + r0[j];
    bool p0 = (sel >> (2 * j)) & 1u, p1 = (sel >> (2 * j + 1)) & 1u;
    if (p0) out[pos] = v0[j];
    if (p1) out[pos + (p0 ? 1 : 0)] = v1[j];
#pragma unroll
    for (int w = 0; w < WAVES; ++w) off += s_cnt[j][w];
  }
}

template <int THREADS, int STRIPES, bool TICKET>
void run_w(const char *name, const int64_t *col, uint64_t n, int64_t k, int64_t *out, uint64_t *dn, void *state,
           int R, unsigned long long *dh) {
  constexpr int TILE = THREADS * 2 * STRIPES;
  uint32_t ntiles = (uint32_t)((n + TILE - 1) / TILE);
  size_t sb = 16 + (size_t)ntiles * 8;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float tot = 0;
  for (int r = 0; r < R + 2; ++r) {
    CK(hipMemsetAsync(state, 0, sb, 0));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((filt_w<THREADS, STRIPES, TICKET>), dim3(ntiles), dim3(THREADS + 64), 0, 0, col, n, k, out, dn,
                       (uint32_t *)state, (uint64_t *)((char *)state + 16), ntiles);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) tot += ms;
  }
  uint64_t cnt;
  CK(hipMemcpy(&cnt, dn, 8, hipMemcpyDeviceToHost));
  CK(hipMemset(dh, 0, 8));
  hipLaunchKernelGGL(checksum, dim3(1024), dim3(256), 0, 0, out, cnt, dh);
  unsigned long long h;
  CK(hipMemcpy(&h, dh, 8, hipMemcpyDeviceToHost));
  double ms = tot / R;
  double gb = (8.0 * n + 8.0 * cnt) / 1e9;
  printf("%-34s %8.4f ms  %7.1f GB/s  count=%llu hash=%016llx\n", name, ms, gb / (ms * 1e-3),
         (unsigned long long)cnt, h);
}

// persistent + ticketed + software-pipelined: a workgroup publishes tile t's aggregate,
// takes its next ticket and issues that tile's loads BEFORE resolving t's look-back, so the
// look-back round trips overlap the next tile's HBM reads.  Wave 0 resolves first and loads
// its share of the next tile afterwards (its vmcnt holds no data loads while it spins).
template <int THREADS, int STRIPES, int OCC>
__global__ __launch_bounds__(THREADS, OCC) void filt_q(const int64_t *__restrict__ col, uint64_t n, int64_t k,
                                                     int64_t *__restrict__ out, uint64_t *__restrict__ out_n,
                                                     uint32_t *__restrict__ ticket, uint64_t *__restrict__ status,
                                                     uint32_t ntiles) {
  constexpr int WAVES = THREADS / kWave;
  constexpr int SROWS = THREADS * 2;
  constexpr int TILE = SROWS * STRIPES;
  __shared__ uint32_t s_cnt[STRIPES][WAVES];
  __shared__ uint32_t s_next;
  __shared__ uint64_t s_excl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  i64x2 cur[STRIPES], nxt[STRIPES];
  auto load = [&](i64x2(&v)[STRIPES], uint32_t t) {
    const uint64_t base = (uint64_t)t * TILE;
    if (base + TILE <= n) {
#pragma unroll
      for (int j = 0; j < STRIPES; ++j)
        v[j] = __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(col + base + j * SROWS + 2 * tid));
    } else {
#pragma unroll
      for (int j = 0; j < STRIPES; ++j) {
        const uint64_t idx = base + j * SROWS + 2 * tid;
        v[j].x = idx < n ? col[idx] : 0;
        v[j].y = idx + 1 < n ? col[idx + 1] : 0;
      }
    }
  };
  if (tid == 0) s_next = atomicAdd(ticket, 1u);
  __syncthreads();
  uint32_t tile = s_next;
  if (tile >= ntiles) return;
  load(cur, tile);
  for (;;) {
    const uint64_t base = (uint64_t)tile * TILE;
    const bool full = base + TILE <= n;
    uint32_t r0[STRIPES];
    uint32_t sel = 0;
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) {
      const uint64_t idx = base + j * SROWS + 2 * tid;
      bool p0 = cur[j].x < k && (full || idx < n);
      bool p1 = cur[j].y < k && (full || idx + 1 < n);
      uint64_t b0 = __ballot(p0), b1 = __ballot(p1);
      r0[j] = lane_rank(b0) + lane_rank(b1);
      sel |= (p0 ? 1u : 0u) << (2 * j);
      sel |= (p1 ? 1u : 0u) << (2 * j + 1);
      if (lane == 0) s_cnt[j][wave] = (uint32_t)(__popcll(b0) + __popcll(b1));
    }
    if (tid == 64) s_next = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tn = s_next;
    if (wave == 0) {
      uint32_t c = 0;
      for (int i = lane; i < STRIPES * WAVES; i += 64) c += (&s_cnt[0][0])[i];
      uint64_t total = wave_sum_u64(c);
      uint64_t excl = lookback<1>(status, tile, total, lane, 1);
      if (lane == 0) {
        s_excl = excl;
        if (tile == ntiles - 1) *out_n = excl + total;
      }
    }
    if (tn < ntiles) load(nxt, tn);
    __syncthreads();
    uint64_t off = s_excl;
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) {
      uint64_t before = 0;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) before += (w < wave) ? s_cnt[j][w] : 0u;
      uint64_t pos = off + before + r0[j];
      bool p0 = (sel >> (2 * j)) & 1u, p1 = (sel >> (2 * j + 1)) & 1u;
      if (p0) out[pos] = cur[j].x;
      if (p1) out[pos + (p0 ? 1 : 0)] = cur[j].y;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) off += s_cnt[j][w];
    }
    if (tn >= ntiles) break;
    tile = tn;
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) cur[j] = nxt[j];
    __syncthreads();
  }
}

// persistent + ticketed, selected values staged in LDS: once a tile is ranked its rows move
// from registers into an LDS buffer (tile-local order), the registers take the NEXT tile's
// loads, and only then is the look-back resolved and the buffer written out with aligned
// 16-B (non-temporal) stores.  The look-back wait overlaps the next tile's HBM reads.
template <int THREADS, int STRIPES, int CAP, bool NTS, int OCC = 1>
__global__ __launch_bounds__(THREADS, OCC) void filt_L(const int64_t *__restrict__ col, uint64_t n, int64_t k,
                                                   int64_t *__restrict__ out, uint64_t *__restrict__ out_n,
                                                   uint32_t *__restrict__ ticket, uint64_t *__restrict__ status,
                                                   uint32_t ntiles) {
  constexpr int WAVES = THREADS / kWave;
  constexpr int SROWS = THREADS * 2;
  constexpr int TILE = SROWS * STRIPES;
  static_assert(STRIPES <= 16, "stripe bases live in lanes 0..15");
  __shared__ int64_t s_buf[CAP];
  __shared__ uint32_t s_cnt[STRIPES][WAVES];
  __shared__ uint32_t s_next;
  __shared__ uint64_t s_excl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  i64x2 v[STRIPES];
  // one code path: 16-B loads at clamped (even) row indices; rows >= n are masked in the rank
  const uint64_t last2 = (n - 2) & ~1ull;  // n >= 2, col 16-B aligned
  auto load = [&](uint32_t t) {
    const uint64_t base = (uint64_t)t * TILE;
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) {
      const uint64_t idx = min(base + j * SROWS + 2 * tid, last2);
      v[j] = __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(col + idx));
    }
  };
if (tid == 0) s_next = atomicAdd(ticket, 1u);
  __syncthreads();
  uint32_t tile = s_next;
  if (tile >= ntiles) return;
  load(tile);
  for (;;) {
    const uint64_t base = (uint64_t)tile * TILE;
    const bool full = base + TILE <= n;
    uint32_t rk[(STRIPES + 3) / 4] = {};  // 7-bit in-wave ranks, 4 per word
    uint32_t sel = 0;
#pragma unroll
    for (int j = 0; j < STRIPES; ++j) {
      const uint64_t idx = base + j * SROWS + 2 * tid;
      bool p0 = v[j].x < k && (full || idx < n);
      bool p1 = v[j].y < k && (full || idx + 1 < n);
      uint64_t b0 = __ballot(p0), b1 = __ballot(p1);
      rk[j / 4] |= (lane_rank(b0) + lane_rank(b1)) << (8 * (j % 4));
      sel |= (p0 ? 1u : 0u) << (2 * j);
      sel |= (p1 ? 1u : 0u) << (2 * j + 1);
      if (lane == 0) s_cnt[j][wave] = (uint32_t)(__popcll(b0) + __popcll(b1));
    }
    if (tid == 64) s_next = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tn = s_next;
    // lane j < STRIPES: stripe j's total (T) and the part before this wave (P); scan T
    uint32_t T = 0, P = 0;
    if (lane < STRIPES) {
#pragma unroll
      for (int w = 0; w < WAVES; ++w) {
        const uint32_t c = s_cnt[lane][w];
        T += c;
        P += w < wave ? c : 0u;
      }
    }
    uint32_t incl = T;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const uint32_t o = __shfl_up(incl, d, 64);
      incl += lane >= d ? o : 0u;
    }
    const uint32_t pre = incl - T + P;  // tile-local start of this wave's rows of stripe `lane`
    const uint32_t total = __builtin_amdgcn_readlane(incl, STRIPES - 1);
    const bool staged = total <= CAP;  // uniform
    auto resolve = [&]() {
      if (wave == 0) {
        uint64_t excl = lookback<1>(status, tile, total, lane, 1);
        if (lane == 0) {
          s_excl = excl;
          if (tile == ntiles - 1) *out_n = excl + total;
        }
      }
    };
    if (staged) {
#pragma unroll
      for (int j = 0; j < STRIPES; ++j) {
        const uint32_t pos = __builtin_amdgcn_readlane(pre, j) + ((rk[j / 4] >> (8 * (j % 4))) & 0xFFu);
        const bool p0 = (sel >> (2 * j)) & 1u, p1 = (sel >> (2 * j + 1)) & 1u;
        if (p0) s_buf[pos] = v[j].x;
        if (p1) s_buf[pos + (p0 ? 1 : 0)] = v[j].y;
      }
    } else {  // more selected rows than the buffer: resolve first, write from registers
      resolve();
      __syncthreads();
      const uint64_t off = s_excl;
#pragma unroll
      for (int j = 0; j < STRIPES; ++j) {
        const uint64_t pos = off + __builtin_amdgcn_readlane(pre, j) + ((rk[j / 4] >> (8 * (j % 4))) & 0xFFu);
        const bool p0 = (sel >> (2 * j)) & 1u, p1 = (sel >> (2 * j + 1)) & 1u;
        if (p0) out[pos] = v[j].x;
        if (p1) out[pos + (p0 ? 1 : 0)] = v[j].y;
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // the registers are free from here on
    if (staged) resolve();              // wave 0 walks before it has data loads in flight
    if (tn < ntiles) load(tn);
    if (staged) {
      __syncthreads();
      const uint64_t excl = s_excl;
      const uint32_t head = (uint32_t)(excl & 1);  // out + excl + head is 16-B aligned
      if (head && tid == 0 && total) out[excl] = s_buf[0];
      for (uint32_t i = head + 2 * tid; i + 1 < total; i += 2 * THREADS) {
        i64x2 w = {s_buf[i], s_buf[i + 1]};
        if (NTS)
          __builtin_nontemporal_store(w, reinterpret_cast<i64x2 *>(out + excl + i));
        else
          *reinterpret_cast<i64x2 *>(out + excl + i) = w;
      }
      if (total > head && ((total - head) & 1) && tid == THREADS - 1) out[excl + total - 1] = s_buf[total - 1];
    }
    if (tn >= ntiles) break;
    tile = tn;
  }
}

template <int THREADS, int STRIPES, int CAP, bool NTS, int OCC = 1>
void run_L(const char *name, const int64_t *col, uint64_t n, int64_t k, int64_t *out, uint64_t *dn, void *state,
           int R, unsigned long long *dh) {
  constexpr int TILE = THREADS * 2 * STRIPES;
  uint32_t ntiles = (uint32_t)((n + TILE - 1) / TILE);
  size_t sb = 16 + (size_t)ntiles * 8;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  int per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, filt_L<THREADS, STRIPES, CAP, NTS, OCC>, THREADS, 0));
  uint32_t grid = (uint32_t)std::min<uint64_t>(ntiles, (uint64_t)prop.multiProcessorCount * per_cu);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float tot = 0;
  for (int r = 0; r < R + 2; ++r) {
    CK(hipMemsetAsync(state, 0, sb, 0));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((filt_L<THREADS, STRIPES, CAP, NTS, OCC>), dim3(grid), dim3(THREADS), 0, 0, col, n, k, out, dn,
                       (uint32_t *)state, (uint64_t *)((char *)state + 16), ntiles);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) tot += ms;
  }
  uint64_t cnt;
  CK(hipMemcpy(&cnt, dn, 8, hipMemcpyDeviceToHost));
  CK(hipMemset(dh, 0, 8));
  hipLaunchKernelGGL(checksum, dim3(1024), dim3(256), 0, 0, out, cnt, dh);
  unsigned long long h;
  CK(hipMemcpy(&h, dh, 8, hipMemcpyDeviceToHost));
  double ms = tot / R;
  double gb = (8.0 * n + 8.0 * cnt) / 1e9;
  printf("%-28s g%-5u %8.4f ms  %7.1f GB/s  count=%llu hash=%016llx\n", name, grid, ms, gb / (ms * 1e-3),
         (unsigned long long)cnt, h);
}

template <int THREADS, int STRIPES, int OCC>
void run_q(const char *name, const int64_t *col, uint64_t n, int64_t k, int64_t *out, uint64_t *dn, void *state,
           int R, unsigned long long *dh, int gridmul) {
  constexpr int TILE = THREADS * 2 * STRIPES;
  uint32_t ntiles = (uint32_t)((n + TILE - 1) / TILE);
  size_t sb = 16 + (size_t)ntiles * 8;
  int per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, filt_q<THREADS, STRIPES, OCC>, THREADS, 0));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  uint32_t grid = (uint32_t)std::min<uint64_t>(ntiles, (uint64_t)per_cu * prop.multiProcessorCount * gridmul / 4);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float tot = 0;
  for (int r = 0; r < R + 2; ++r) {
    CK(hipMemsetAsync(state, 0, sb, 0));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((filt_q<THREADS, STRIPES, OCC>), dim3(grid), dim3(THREADS), 0, 0, col, n, k, out, dn,
                       (uint32_t *)state, (uint64_t *)((char *)state + 16), ntiles);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) tot += ms;
  }
  uint64_t cnt;
  CK(hipMemcpy(&cnt, dn, 8, hipMemcpyDeviceToHost));
  CK(hipMemset(dh, 0, 8));
  hipLaunchKernelGGL(checksum, dim3(1024), dim3(256), 0, 0, out, cnt, dh);
  unsigned long long h;
  CK(hipMemcpy(&h, dh, 8, hipMemcpyDeviceToHost));
  double ms = tot / R;
  double gb = (8.0 * n + 8.0 * cnt) / 1e9;
  printf("%-28s occ%d g%-5u %8.4f ms  %7.1f GB/s  count=%llu hash=%016llx\n", name, per_cu, grid, ms,
         gb / (ms * 1e-3), (unsigned long long)cnt, h);
}

int main(int argc, char **argv) {
  setvbuf(stdout, NULL, _IONBF, 0);
  uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 100000000ull;
  double s = argc > 2 ? atof(argv[2]) : 0.5;
  int R = 20;
  int64_t k = (int64_t)(s * 4611686018427387904.0);
  int64_t *col, *out;
  uint64_t *dn;
  void *state;
  unsigned long long *dh;
  CK(hipMalloc(&col, n * 8));
  CK(hipMalloc(&out, n * 8));
  CK(hipMalloc(&dn, 64));
  CK(hipMalloc(&dh, 64));
  CK(hipMalloc(&state, 16 + (n / 256 + 16) * 8));
  hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, 0, col, n);
  CK(hipDeviceSynchronize());
  if (argc > 3 && atoi(argv[3]) != 99 && atoi(argv[3]) != 98) goto variants;
  if (argc > 3 && atoi(argv[3]) == 98) goto copies;
  {  // reference copy bandwidth: read n*8, write n*4 (half)
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float tot = 0;
    for (int r = 0; r < R + 2; ++r) {
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(copyk, dim3(8192), dim3(256), 0, 0, col, out, n);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r >= 2) tot += ms;
    }
    double ms = tot / R;
    printf("%-34s %8.4f ms  %7.1f GB/s\n", "copy read n, write n/2", ms, 12.0 * n / 1e9 / (ms * 1e-3));
  }
  {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int grid : {1024, 2048, 4096, 8192}) {
      float tot = 0;
      for (int r = 0; r < R + 2; ++r) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(copy4, dim3(grid), dim3(256), 0, 0, col, out, n);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 2) tot += ms;
      }
      double ms = tot / R;
      printf("copy4 grid %-5d                   %8.4f ms  %7.1f GB/s\n", grid, ms, 12.0 * n / 1e9 / (ms * 1e-3));
    }
  }
copies:
  if (argc > 3 && atoi(argv[3]) == 98) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto T = [&](const char *nm, void (*kf)(const int64_t *, int64_t *, uint64_t), int grid) {
      float tot = 0;
      for (int r = 0; r < R + 2; ++r) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(kf, dim3(grid), dim3(256), 0, 0, col, out, n);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 2) tot += ms;
      }
      double ms = tot / R;
      printf("%-22s grid %-5d %8.4f ms  %7.1f GB/s\n", nm, grid, ms, 12.0 * n / 1e9 / (ms * 1e-3));
    };
    for (int grid : {1024, 2048, 4096}) {
      T("copyN 4", copyN<4, false, false>, grid);
      T("copyN 4 NTL", copyN<4, true, false>, grid);
      T("copyN 4 NTL NTS", copyN<4, true, true>, grid);
      T("copyN 8 NTL", copyN<8, true, false>, grid);
      T("copyN 8 NTL NTS", copyN<8, true, true>, grid);
      T("copyN 16 NTL", copyN<16, true, false>, grid);
      T("copyN 16 NTL NTS", copyN<16, true, true>, grid);
    }
    return 0;
  }
variants:
  int v = argc > 3 ? atoi(argv[3]) : -1;
  int idx = 0;
  if (v < 0 || v == idx) run<512, 16, false, false, 1, false>("512x16 noticket", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 16, false, false, 1, false, 4>("512x16 noticket LB4", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 16, false, true, 1, false>("512x16 noticket NT", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<768, 16, false, false, 1, false>("768x16 noticket", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<1024, 16, false, false, 1, false>("1024x16 noticket", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 12, false, false, 1, false>("512x12 noticket", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<384, 16, false, false, 1, false>("384x16 noticket", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 16, false, false, 0, false>("512x16 noticket nosleep", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 16, true, false, 1, false>("512x16 LDS noticket", col, n, k, out, dn, state, R, dh);
  ++idx;
  // 9: the product kernel's scheme (ticket + NT)
  if (v < 0 || v == idx) run<512, 16, false, true, 1, true>("512x16 ticket NT (product)", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 16, false, true, 1, false, 1, 1>("NT nolookback", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 16, false, true, 1, false, 1, 2>("NT nowrite", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 16, false, true, 1, false, 1, 3>("NT read+rank only", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<256, 16, false, true, 1, false, 1, 3>("256x16 NT read+rank only", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<256, 8, false, true, 1, false, 1, 3>("256x8 NT read+rank only", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<256, 8, false, true, 1, false, 1, 1>("256x8 NT nolookback", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 16, false, true, 1, true, 1, 0, true>("product + NTS", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 16, false, true, 1, false, 1, 1, true>("nolookback NTS", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<256, 8, false, true, 1, false>("256x8 noticket NT", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<256, 16, false, true, 1, false>("256x16 noticket NT", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<512, 8, false, true, 1, false>("512x8 noticket NT", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run<256, 16, false, true, 1, false, 1, 0, true>("256x16 noticket NT NTS", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run_L<1024, 16, 18944, true>("L 1024x16 NTS", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run_L<1024, 16, 18944, false>("L 1024x16", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run_L<1024, 8, 18944, true>("L 1024x8 NTS", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run_L<512, 16, 18944, true>("L 512x16 NTS", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run_L<512, 16, 9984, true, 2>("L 512x16 cap9984 occ2 NTS", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run_L<256, 16, 4992, true, 4>("L 256x16 cap4992 occ4 NTS", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run_L<1024, 16, 20224, true>("L 1024x16 cap20224 NTS", col, n, k, out, dn, state, R, dh);
  ++idx;
  if (v < 0 || v == idx) run_q<512, 16, 1>("q 512x16 occ1", col, n, k, out, dn, state, R, dh, 4);
  ++idx;
  if (v < 0 || v == idx) run_q<512, 8, 2>("q 512x8 occ2", col, n, k, out, dn, state, R, dh, 4);
  ++idx;
  if (v < 0 || v == idx) run_q<1024, 8, 1>("q 1024x8 occ1", col, n, k, out, dn, state, R, dh, 4);
  ++idx;
  if (v < 0 || v == idx) run_q<256, 16, 2>("q 256x16 occ2", col, n, k, out, dn, state, R, dh, 4);
  ++idx;
  if (v < 0 || v == idx) run_q<512, 12, 1>("q 512x12 occ1", col, n, k, out, dn, state, R, dh, 4);
  ++idx;
  if (v < 0 || v == idx) run_q<512, 16, 1>("q 512x16 occ1 grid x2", col, n, k, out, dn, state, R, dh, 8);
  ++idx;
  if (v < 0 || v == idx) run_p<512, 16, true, 1>("p 512x16 NT", col, n, k, out, dn, state, R, dh, 4);
  ++idx;
  if (v < 0 || v == idx) run_w<512, 16, true>("w 512x16 ticket", col, n, k, out, dn, state, R, dh);
  ++idx;
  return 0;
}
