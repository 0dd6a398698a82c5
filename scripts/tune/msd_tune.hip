// msd_tune.hip — standalone variant sweep for the MSD sort's scatter level and local sort
// (not product code; the product kernels live in nutdb_amd/csrc/msd_sort.hip).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/tune/msd_tune.hip -o scripts/tune/bin/msd_tune
// run:   msd_tune            (1.25e9 random keys; prints ms per variant)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../../nutdb_amd/csrc/common.hpp"

using namespace nut;

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));   \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

constexpr int BINS = 256;

__global__ void gen(uint64_t *c, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c[i] = gen_u64(0x50, i);
}

// ------------------------------------------------------------------ scatter variants
// MODE bits: 1 = cursor by plain load (no atomic; output invalid) , 2 = direct scatter (no LDS staging)
template <int THREADS, int ITEMS, int MODE>
__global__ __launch_bounds__(THREADS) void scatter(const uint64_t *__restrict__ src, uint64_t *__restrict__ dst, uint64_t n,
                                                   int shift, unsigned long long *__restrict__ cursor) {
  constexpr int TILE = THREADS * ITEMS;
  constexpr bool STAGE = !(MODE & 2);
  __shared__ uint64_t s_keys[STAGE ? TILE : 1];
  __shared__ uint32_t s_cnt[BINS];
  __shared__ uint32_t s_tex[BINS];
  __shared__ uint64_t s_gb[BINS];
  __shared__ uint32_t s_wsum[BINS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < BINS; i += THREADS) s_cnt[i] = 0;
  const uint64_t lo = (uint64_t)blockIdx.x * TILE;
  const uint32_t cnt = (uint32_t)min<uint64_t>(TILE, n - lo);
  const uint64_t *s = src + lo;
  uint64_t key[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const uint32_t idx = (uint32_t)i * THREADS + tid;
    key[i] = idx < cnt ? __builtin_nontemporal_load(s + idx) : 0;
  }
  __syncthreads();
  uint32_t rk[ITEMS];
#pragma unroll
  for (int i = 0; i < ITEMS; ++i) {
    const uint32_t idx = (uint32_t)i * THREADS + tid;
    rk[i] = idx < cnt ? atomicAdd(&s_cnt[(key[i] >> shift) & 255], 1u) : 0u;
  }
  __syncthreads();
  uint32_t c = 0, incl = 0;
  if (tid < BINS) {
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
  if (tid < BINS) {
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < BINS / 64; ++w) add += (w < wave) ? s_wsum[w] : 0u;
    const uint32_t tex = incl - c + add;
    s_tex[tid] = tex;
    // MODE 1: plain load of the cursor and sequential output (measures the atomic and the
    // scattered-run write pattern together)
    const uint64_t gb = (MODE & 1) ? cursor[tid] : (c ? (uint64_t)atomicAdd(&cursor[tid], (unsigned long long)c) : 0);
    s_gb[tid] = STAGE ? gb - tex : gb;
  }
  __syncthreads();
  if (STAGE) {
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t idx = (uint32_t)i * THREADS + tid;
      if (idx < cnt) s_keys[s_tex[(key[i] >> shift) & 255] + rk[i]] = key[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t j = (uint32_t)i * THREADS + tid;
      if (j < cnt) {
        const uint64_t k = s_keys[j];
        uint64_t p = s_gb[(k >> shift) & 255] + j;
        if (MODE & 1) p = lo + j;
        dst[p] = k;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t idx = (uint32_t)i * THREADS + tid;
      if (idx < cnt) {
        uint64_t p = s_gb[(key[i] >> shift) & 255] + rk[i];
        if (MODE & 1) p = lo + idx;
        dst[p] = key[i];
      }
    }
  }
}

// ------------------------------------------------------------------ local sort: product kernels
#define NUT_MSD_KERNELS_ONLY
#define NUT_MSD_PROFILE_STOP
#include "../../nutdb_amd/csrc/msd_sort.hip"

__global__ void gen48(uint64_t *c, uint64_t n) {  // segment keys share their top 16 bits
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c[i] = gen_u64(0x50, i) & ((1ull << 48) - 1);
}

template <int MODE>
__global__ void check_sorted(const uint64_t *d, uint64_t n, uint32_t seglen, int bits, unsigned long long *bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if ((i + 1) % seglen == 0) continue;
    const uint64_t m = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    if ((d[i] & m) > (d[i + 1] & m)) atomicAdd(bad, 1ull);
  }
}

static float time_it(hipEvent_t a, hipEvent_t b) {
  float ms;
  CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

template <int T, int K, bool PF>
static void local_sweep(nut::MsBufs bf, uint64_t *a, uint64_t *b, uint64_t n, uint32_t seglen, hipEvent_t e0,
                        hipEvent_t e1, unsigned long long *bad) {
  const uint64_t nseg = n / seglen;
  std::vector<nut::MsSeg> segs(nseg);
  std::vector<uint32_t> fb(nseg + 1);
  fb[0] = (uint32_t)nseg;
  for (uint64_t i = 0; i < nseg; ++i) {
    segs[i] = nut::MsSeg{i * seglen, seglen, 2, 48};  // keys share their top 16 bits
    fb[1 + i] = (uint32_t)i;
  }
  nut::MsSeg *dseg;
  uint32_t *dfb, *dfb0;
  CK(hipMalloc(&dseg, nseg * sizeof(nut::MsSeg)));
  CK(hipMalloc(&dfb, (nseg + 1) * 4));
  CK(hipMalloc(&dfb0, (nseg + 1) * 4));
  CK(hipMemcpy(dseg, segs.data(), nseg * sizeof(nut::MsSeg), hipMemcpyHostToDevice));
  CK(hipMemcpy(dfb, fb.data(), (nseg + 1) * 4, hipMemcpyHostToDevice));
  int per_cu = 1, ncu = 256;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nut::ms_local_kernel<T, K, PF>, T, 0));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned grid = PF ? (unsigned)std::min<uint64_t>(nseg, (uint64_t)ncu * per_cu) : (unsigned)nseg;
  printf("local<%d,%d,%d>: %d workgroups per CU, grid %u\n", T, K, (int)PF, per_cu, grid);
  const int stops[] = {0, 1, 3, 4, 5, 0};
  for (int variant = 0; variant < 6; ++variant) {
    const int stop = stops[variant];
    CK(hipMemcpyToSymbol(HIP_SYMBOL(nut::g_ms_stop), &stop, sizeof(int)));
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
      hipLaunchKernelGGL(gen48, dim3(4096), dim3(256), 0, 0, b, n);
      CK(hipMemset(dfb0, 0, 4));
      CK(hipEventRecord(e0));
      if (variant < 5)
        hipLaunchKernelGGL((nut::ms_local_kernel<T, K, PF>), dim3(grid), dim3(T), 0, 0, bf,
                           (const nut::MsSeg *)dseg, (uint32_t)nseg, 0ull, 0ull, dfb0);
      else
        hipLaunchKernelGGL((nut::ms_lsd_kernel<T, K>), dim3((unsigned)nseg), dim3(T), 0, 0, bf,
                           (const nut::MsSeg *)dseg, 0ull, 0ull, (const uint32_t *)dfb);
      CK(hipEventRecord(e1));
      best = std::min(best, time_it(e0, e1));
    }
    uint32_t nfb = 0;
    CK(hipMemcpy(&nfb, dfb0, 4, hipMemcpyDeviceToHost));
    CK(hipMemset(bad, 0, 8));
    hipLaunchKernelGGL(check_sorted<0>, dim3(4096), dim3(256), 0, 0, a, nseg * seglen, seglen, 64, bad);
    unsigned long long hb;
    CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    printf("local<%d,%d> %s stop=%d seglen=%u: %.3f ms  (%.0f GB/s) unsorted pairs %llu fallbacks %u\n", T, K,
           variant < 5 ? "msd+net" : "lsd-ballot", stop, seglen, best, 16.0 * nseg * seglen / best / 1e6, hb,
           variant < 5 ? nfb : 0u);
  }
  CK(hipFree(dseg));
  CK(hipFree(dfb));
  CK(hipFree(dfb0));
}

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1250000000ull;
  uint64_t *a, *b;
  unsigned long long *cur, *bad;
  CK(hipMalloc(&a, n * 8));
  CK(hipMalloc(&b, (n + (1u << 22)) * 8));  // slack: digit counts vary around n / 256
  CK(hipMalloc(&cur, BINS * 8 * 4));
  CK(hipMalloc(&bad, 8));
  hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, 0, a, n);
  // cursors: digit 7 of uniform keys -> n/256 each
  std::vector<unsigned long long> hc(BINS);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto reset_cur = [&]() {
    // exact digit bases need a histogram; approximate starts are fine for timing, but
    // keep writes in bounds: base d = d * (n / 256) - slack handled by clamping tiles
    for (int d = 0; d < BINS; ++d) hc[d] = (unsigned long long)d * (n / BINS);
    CK(hipMemcpy(cur, hc.data(), BINS * 8, hipMemcpyHostToDevice));
  };
#define RUN_SCATTER(T, I, M)                                                                      \
  {                                                                                               \
    float best = 1e9;                                                                             \
    for (int r = 0; r < 3; ++r) {                                                                 \
      reset_cur();                                                                                \
      CK(hipEventRecord(e0));                                                                     \
      hipLaunchKernelGGL((scatter<T, I, M>), dim3((unsigned)((n + T * I - 1) / (T * I))), dim3(T), 0, 0, a, b, \
                         n, 56, cur);                                                              \
      CK(hipEventRecord(e1));                                                                     \
      best = std::min(best, time_it(e0, e1));                                                     \
    }                                                                                             \
    printf("scatter T=%d I=%d mode=%d: %.3f ms  (%.0f GB/s)\n", T, I, M, best, 16.0 * n / best / 1e6); \
  }
  // cursors start at d * n/256 (uniform keys): runs land where the real level puts them
  RUN_SCATTER(512, 16, 0);
  RUN_SCATTER(512, 16, 1);
  RUN_SCATTER(512, 16, 2);
  RUN_SCATTER(256, 16, 0);
  RUN_SCATTER(1024, 16, 0);
  RUN_SCATTER(512, 8, 0);

  nut::MsBufs bf{nullptr, a, b};  // in unused, a = out, b = tmp (segment source)
  const uint32_t seglen = argc > 2 ? (uint32_t)atoi(argv[2]) : 4768;
  if (seglen <= 6144) local_sweep<512, 12, true>(bf, a, b, n, seglen, e0, e1, bad);
  else local_sweep<1024, 24, false>(bf, a, b, n, seglen, e0, e1, bad);
  return 0;
}
