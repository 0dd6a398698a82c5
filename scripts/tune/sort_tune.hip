// sort_tune.hip — standalone variant sweep for one onesweep radix pass (not product code).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/tune/sort_tune.hip -o scripts/tune/bin/sort_tune
// run:   sort_tune N VARIANT      (one pass over N random keys, digit = bits 0..7)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../../nutdb_amd/csrc/common.hpp"

using namespace nut;

constexpr int BINS = 256;
constexpr uint64_t AGG = 1ull << 62, INC = 2ull << 62, VAL = (1ull << 62) - 1;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));            \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ uint64_t peers8(uint32_t d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint64_t bb = __ballot((d >> b) & 1u);
    m &= ((d >> b) & 1u) ? bb : ~bb;
  }
  return m;
}

// MODE bits: 1 = no look-back, 2 = no LDS staging (direct scatter), 4 = unstable LDS-atomic rank,
//            8 = 16-B loads (2 keys per lane per item pair)
template <int THREADS, int ITEMS, int MODE, int LBW>
__global__ __launch_bounds__(THREADS) void pass(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t n,
                                                int shift, const uint64_t *__restrict__ dbase,
                                                uint64_t *__restrict__ status, unsigned long long *__restrict__ steps_hist) {
  constexpr int WAVES = THREADS / kWave;
  constexpr int TILE = THREADS * ITEMS;
  constexpr bool STAGE = !(MODE & 2);
  __shared__ uint64_t s_keys[STAGE ? TILE : 1];
  __shared__ uint32_t s_wcnt[WAVES][BINS];
  __shared__ uint32_t s_tex[BINS];
  __shared__ uint64_t s_gbase[BINS];
  __shared__ uint32_t s_wsum[BINS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < WAVES * BINS; i += THREADS) (&s_wcnt[0][0])[i] = 0;
  const uint32_t tile = blockIdx.x;
  const uint64_t tbase = (uint64_t)tile * TILE;
  const uint64_t wbase = tbase + (uint64_t)wave * ITEMS * kWave;
  uint64_t key[ITEMS];
  uint32_t rank[ITEMS];
  if (MODE & 8) {
#pragma unroll
    for (int i = 0; i < ITEMS; i += 2) {
      const uint64_t idx = wbase + (uint64_t)i * kWave + 2 * lane;
      if (idx + 1 < n) {
        u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(in + idx));
        key[i] = v.x;
        key[i + 1] = v.y;
      } else {
        key[i] = idx < n ? in[idx] : 0;
        key[i + 1] = 0;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint64_t idx = wbase + (uint64_t)i * kWave + lane;
      key[i] = idx < n ? in[idx] : 0;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const uint64_t idx = (MODE & 8) ? wbase + (uint64_t)(i & ~1) * kWave + 2 * lane + (i & 1)
                                    : wbase + (uint64_t)i * kWave + lane;
    const bool valid = idx < n;
    const uint32_t d = (uint32_t)(key[i] >> shift) & 255u;
    if (MODE & 4) {
      rank[i] = valid ? atomicAdd(&s_wcnt[wave][d], 1u) : 0u;
    } else {
      const uint64_t pe = peers8(d, valid);
      const uint32_t before = lane_rank(pe);
      const uint32_t cnt = (uint32_t)__popcll(pe);
      uint32_t prior = valid ? s_wcnt[wave][d] : 0u;
      rank[i] = prior + before;
      if (valid && before == 0) s_wcnt[wave][d] = prior + cnt;
    }
  }
  __syncthreads();
  for (int d = tid; d < BINS; d += THREADS) {
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
      const uint32_t c = s_wcnt[w][d];
      s_wcnt[w][d] = tot;
      tot += c;
    }
    s_tex[d] = tot;  // temporarily the tile count
  }
  __syncthreads();
  uint32_t v = 0, tot = 0;
  if (tid < BINS) {
    tot = s_tex[tid];
    v = tot;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      uint32_t y = __shfl_up(v, off, 64);
      if (lane >= off) v += y;
    }
    if (lane == 63) s_wsum[wave] = v;
  }
  __syncthreads();
  if (tid < BINS) {
    const int d = tid;
    uint32_t add = 0;
    for (int w = 0; w < (BINS / 64); ++w) add += (w < wave) ? s_wsum[w] : 0u;
    const uint32_t tex = v - tot + add;
    uint64_t excl = 0;
    uint64_t *my = &status[(uint64_t)tile * BINS + d];
    if (!(MODE & 1)) {
      if (tile == 0) {
        st_agent(my, INC | tot);
      } else {
        st_agent(my, AGG | tot);
        int64_t j = (int64_t)tile - 1;
        bool done = false;
        uint32_t steps = 0, waits = 0;
        while (!done) {
          ++steps;
          uint64_t sv[LBW];
#pragma unroll
          for (int m = 0; m < LBW; ++m) sv[m] = j - m >= 0 ? ld_agent(&status[(uint64_t)(j - m) * BINS + d]) : INC;
#pragma unroll
          for (int m = 0; m < LBW; ++m) {
            if (done) break;
            uint64_t sm = sv[m];
            while ((sm >> 62) == 0) {
              __builtin_amdgcn_s_sleep(1);
              ++waits;
              sm = ld_agent(&status[(uint64_t)(j - m) * BINS + d]);
            }
            excl += sm & VAL;
            if ((sm >> 62) == 2) done = true;
          }
          j -= LBW;
        }
        st_agent(my, INC | (excl + tot));
        if (d == 0 && steps_hist) {
          atomicAdd(&steps_hist[min(steps, 63u)], 1ull);
          atomicAdd(&steps_hist[64 + min(waits, 63u)], 1ull);
        }
      }
    }
    s_gbase[d] = dbase[d] + excl;
    s_tex[d] = tex;
  }
  __syncthreads();
  if (STAGE) {
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint64_t idx = (MODE & 8) ? wbase + (uint64_t)(i & ~1) * kWave + 2 * lane + (i & 1)
                                      : wbase + (uint64_t)i * kWave + lane;
      if (idx < n) {
        const uint32_t dd = (uint32_t)(key[i] >> shift) & 255u;
        s_keys[s_tex[dd] + s_wcnt[wave][dd] + rank[i]] = key[i];
      }
    }
    __syncthreads();
    const uint32_t valid_n = (uint32_t)min<uint64_t>(TILE, n - tbase);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t j = (uint32_t)i * THREADS + tid;
      if (j < valid_n) {
        const uint64_t k = s_keys[j];
        const uint32_t dd = (uint32_t)(k >> shift) & 255u;
        out[s_gbase[dd] + (j - s_tex[dd])] = k;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint64_t idx = (MODE & 8) ? wbase + (uint64_t)(i & ~1) * kWave + 2 * lane + (i & 1)
                                      : wbase + (uint64_t)i * kWave + lane;
      if (idx < n) {
        const uint32_t dd = (uint32_t)(key[i] >> shift) & 255u;
        out[s_gbase[dd] + s_tex[dd] - s_tex[dd] + s_wcnt[wave][dd] + rank[i] + 0] = key[i];
      }
    }
  }
}

__global__ void gen(uint64_t *c, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c[i] = gen_u64(0x50, i);
}

__global__ void hist0(const uint64_t *in, uint64_t n, unsigned long long *h) {
  __shared__ uint32_t s[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s[i] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&s[in[i] & 255], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x) atomicAdd(&h[i], (unsigned long long)s[i]);
}

__global__ void check(const uint64_t *o, uint64_t n, unsigned long long *bad) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x + 1; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if ((o[i] & 255) < (o[i - 1] & 255)) atomicAdd(bad, 1ull);
}

unsigned long long *g_steps = nullptr;

template <int THREADS, int ITEMS, int MODE, int LBW>
void run(const char *name, const uint64_t *in, uint64_t *out, uint64_t n, const uint64_t *dbase, uint64_t *status,
         unsigned long long *bad) {
  constexpr int TILE = THREADS * ITEMS;
  uint64_t ntiles = (n + TILE - 1) / TILE;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float tot = 0;
  const int R = 10;
  for (int r = 0; r < R + 2; ++r) {
    CK(hipMemsetAsync(status, 0, ntiles * BINS * 8, 0));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((pass<THREADS, ITEMS, MODE, LBW>), dim3((unsigned)ntiles), dim3(THREADS), 0, 0, in, out, n, 0,
                       dbase, status, r == R + 1 ? g_steps : nullptr);
    CK(hipGetLastError());
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) tot += ms;
  }
  CK(hipMemset(bad, 0, 8));
  hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, out, n, bad);
  unsigned long long hb;
  CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  double ms = tot / R;
  printf("%-36s %8.3f ms  %7.1f GB/s  unsorted=%llu\n", name, ms, 16.0 * n / 1e9 / (ms * 1e-3), hb);
  unsigned long long hs[128];
  CK(hipMemcpy(hs, g_steps, sizeof hs, hipMemcpyDeviceToHost));
  printf("  walk steps:");
  for (int i = 0; i < 64; ++i) if (hs[i]) printf(" %d:%llu", i, hs[i]);
  printf("\n  wait polls:");
  for (int i = 64; i < 128; ++i) if (hs[i]) printf(" %d:%llu", i - 64, hs[i]);
  printf("\n");
  CK(hipMemset(g_steps, 0, sizeof hs));
}

// SUB sub-tiles of THREADS*ITEMS keys per workgroup: one look-back per SUB*THREADS*ITEMS
// keys; ranks run across the sub-tiles; staging in LDS one sub-tile of positions at a time.
template <int THREADS, int ITEMS, int SUB>
__global__ __launch_bounds__(THREADS) void pass2(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t n,
                                                 int shift, const uint64_t *__restrict__ dbase,
                                                 uint64_t *__restrict__ status, uint32_t *__restrict__ ticket) {
  constexpr int WAVES = THREADS / kWave;
  constexpr int STILE = THREADS * ITEMS;
  constexpr int TILE = STILE * SUB;
  __shared__ uint64_t s_keys[STILE];
  __shared__ uint32_t s_wcnt[WAVES][BINS];
  __shared__ uint32_t s_tex[BINS];
  __shared__ uint64_t s_gbase[BINS];
  __shared__ uint32_t s_wsum[BINS / 64];
  __shared__ uint32_t s_tile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < WAVES * BINS; i += THREADS) (&s_wcnt[0][0])[i] = 0;
  if (tid == 0) s_tile = atomicAdd(ticket, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t tbase = (uint64_t)tile * TILE;
  uint64_t key[SUB][ITEMS];
  uint32_t rank[SUB][ITEMS];
#pragma unroll
  for (int sb = 0; sb < SUB; ++sb) {
    const uint64_t wbase = tbase + (uint64_t)sb * STILE + (uint64_t)wave * ITEMS * kWave;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint64_t idx = wbase + (uint64_t)i * kWave + lane;
      key[sb][i] = idx < n ? in[idx] : 0;
    }
  }
#pragma unroll
  for (int sb = 0; sb < SUB; ++sb) {
    const uint64_t wbase = tbase + (uint64_t)sb * STILE + (uint64_t)wave * ITEMS * kWave;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint64_t idx = wbase + (uint64_t)i * kWave + lane;
      const bool valid = idx < n;
      const uint32_t d = (uint32_t)(key[sb][i] >> shift) & 255u;
      const uint64_t pe = peers8(d, valid);
      const uint32_t before = lane_rank(pe);
      const uint32_t cnt = (uint32_t)__popcll(pe);
      uint32_t prior = valid ? s_wcnt[wave][d] : 0u;
      rank[sb][i] = prior + before;
      if (valid && before == 0) s_wcnt[wave][d] = prior + cnt;
    }
  }
  __syncthreads();
  uint32_t v = 0, tot = 0;
  if (tid < BINS) {
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
      const uint32_t c = s_wcnt[w][tid];
      s_wcnt[w][tid] = tot;
      tot += c;
    }
    v = tot;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      uint32_t y = __shfl_up(v, off, 64);
      if (lane >= off) v += y;
    }
    if (lane == 63) s_wsum[wave] = v;
  }
  __syncthreads();
  if (tid < BINS) {
    const int d = tid;
    uint32_t add = 0;
    for (int w = 0; w < (BINS / 64); ++w) add += (w < wave) ? s_wsum[w] : 0u;
    s_tex[d] = v - tot + add;
    uint64_t excl = 0;
    uint64_t *my = &status[(uint64_t)tile * BINS + d];
    if (tile == 0) {
      st_agent(my, INC | tot);
    } else {
      st_agent(my, AGG | tot);
      int64_t j = (int64_t)tile - 1;
      for (;;) {
        uint64_t sm = ld_agent(&status[(uint64_t)j * BINS + d]);
        while ((sm >> 62) == 0) {
          __builtin_amdgcn_s_sleep(1);
          sm = ld_agent(&status[(uint64_t)j * BINS + d]);
        }
        excl += sm & VAL;
        if ((sm >> 62) == 2) break;
        --j;
      }
      st_agent(my, INC | (excl + tot));
    }
    s_gbase[d] = dbase[d] + excl;
  }
  __syncthreads();
  const uint32_t valid_n = (uint32_t)min<uint64_t>(TILE, n - min<uint64_t>(n, tbase));
#pragma unroll
  for (int half = 0; half < SUB; ++half) {
    const uint32_t lo = (uint32_t)half * STILE, hi = lo + STILE;
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb) {
      const uint64_t wbase = tbase + (uint64_t)sb * STILE + (uint64_t)wave * ITEMS * kWave;
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const uint64_t idx = wbase + (uint64_t)i * kWave + lane;
        if (idx < n) {
          const uint32_t dd = (uint32_t)(key[sb][i] >> shift) & 255u;
          const uint32_t pos = s_tex[dd] + s_wcnt[wave][dd] + rank[sb][i];
          if (pos >= lo && pos < hi) s_keys[pos - lo] = key[sb][i];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t j = lo + (uint32_t)i * THREADS + tid;
      if (j < valid_n) {
        const uint64_t k = s_keys[j - lo];
        const uint32_t dd = (uint32_t)(k >> shift) & 255u;
        out[s_gbase[dd] + (j - s_tex[dd])] = k;
      }
    }
    __syncthreads();
  }
}

template <int THREADS, int ITEMS, int SUB>
void run2(const char *name, const uint64_t *in, uint64_t *out, uint64_t n, const uint64_t *dbase, uint64_t *status,
          unsigned long long *bad, uint32_t *ticket) {
  constexpr int TILE = THREADS * ITEMS * SUB;
  uint64_t ntiles = (n + TILE - 1) / TILE;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float tot = 0;
  const int R = 10;
  for (int r = 0; r < R + 2; ++r) {
    CK(hipMemsetAsync(status, 0, ntiles * BINS * 8, 0));
    CK(hipMemsetAsync(ticket, 0, 4, 0));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((pass2<THREADS, ITEMS, SUB>), dim3((unsigned)ntiles), dim3(THREADS), 0, 0, in, out, n, 0, dbase,
                       status, ticket);
    CK(hipGetLastError());
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2) tot += ms;
  }
  CK(hipMemset(bad, 0, 8));
  hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, out, n, bad);
  unsigned long long hb;
  CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  double ms = tot / R;
  printf("%-36s %8.3f ms  %7.1f GB/s  unsorted=%llu\n", name, ms, 16.0 * n / 1e9 / (ms * 1e-3), hb);
}

int main(int argc, char **argv) {
  setvbuf(stdout, NULL, _IONBF, 0);
  uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 250000000ull;
  int v = argc > 2 ? atoi(argv[2]) : 0;
  uint64_t *in, *out, *status, *dbase;
  unsigned long long *h, *bad;
  CK(hipMalloc(&in, n * 8));
  CK(hipMalloc(&out, n * 8 + (1 << 20)));
  CK(hipMalloc(&status, (n / 1024 + 16) * BINS * 8));
  CK(hipMalloc(&dbase, BINS * 8));
  CK(hipMalloc(&h, BINS * 8));
  CK(hipMalloc(&bad, 8));
  CK(hipMalloc(&g_steps, 128 * 8));
  CK(hipMemset(g_steps, 0, 128 * 8));
  hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, 0, in, n);
  CK(hipMemset(h, 0, BINS * 8));
  hipLaunchKernelGGL(hist0, dim3(2048), dim3(256), 0, 0, in, n, h);
  std::vector<unsigned long long> hh(BINS);
  CK(hipMemcpy(hh.data(), h, BINS * 8, hipMemcpyDeviceToHost));
  std::vector<uint64_t> base(BINS);
  uint64_t run_ = 0;
  for (int i = 0; i < BINS; ++i) {
    base[i] = run_;
    run_ += hh[i];
  }
  CK(hipMemcpy(dbase, base.data(), BINS * 8, hipMemcpyHostToDevice));
  int idx = 0;
#define V(...) \
  if (v == idx++) run<__VA_ARGS__>
  uint32_t *ticket;
  CK(hipMalloc(&ticket, 64));
#define V2(...) \
  if (v == idx++) run2<__VA_ARGS__>
  V2(512, 16, 1)("T 512x16 sub1", in, out, n, dbase, status, bad, ticket);
  V2(512, 16, 2)("T 512x16 sub2", in, out, n, dbase, status, bad, ticket);
  V2(512, 8, 2)("T 512x8 sub2", in, out, n, dbase, status, bad, ticket);
  V2(512, 8, 4)("T 512x8 sub4", in, out, n, dbase, status, bad, ticket);
  V2(256, 16, 2)("T 256x16 sub2", in, out, n, dbase, status, bad, ticket);
  V2(512, 12, 2)("T 512x12 sub2", in, out, n, dbase, status, bad, ticket);
  V2(1024, 8, 2)("T 1024x8 sub2", in, out, n, dbase, status, bad, ticket);
  return 0;
}
