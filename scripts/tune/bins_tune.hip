// bins_tune.hip — what an exact key scatter costs as its bin count grows (not product code).
// Question (r4 verdict item 2): at P ranks, folding the sample sort's range
// partition into the receiver's level 0 means one sender scatter into P x 512 buckets
// instead of a P-bin scatter followed by the receiver's 512-bin level.  This harness times
// one LDS-staged exact scatter of 8-B keys (per-tile digit ranks in LDS, one global cursor
// atomic per digit and tile, staging in digit order, coalesced write-out of each digit's
// run) at 8, 512, 1024, 4096 bins over the same 1.25e9 keys, next to a copy of the keys.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/tune/bins_tune.hip -o scripts/tune/bin/bins_tune
// run:   bins_tune [keys]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../../nutdb_amd/csrc/common.hpp"

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                                      \
    }                                                               \
  } while (0)

__global__ void gen_keys(uint64_t *k, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    k[i] = nut::gen_u64(0x5EED, i);
}

template <int BITS>
__global__ void hist_kernel(const uint64_t *k, uint64_t n, unsigned long long *h) {
  constexpr int B = 1 << BITS;
  __shared__ uint32_t c[B];
  for (int i = threadIdx.x; i < B; i += blockDim.x) c[i] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&c[k[i] >> (64 - BITS)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < B; i += blockDim.x)
    if (c[i]) atomicAdd(&h[i], (unsigned long long)c[i]);
}

// sum of mix64(key) and the out-of-order neighbours (digit decreases) of the output
__global__ void check_kernel(const uint64_t *o, uint64_t n, int bits, unsigned long long *r) {
  unsigned long long h = 0, bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    h += nut::mix64(o[i]);
    if (i && (o[i] >> (64 - bits)) < (o[i - 1] >> (64 - bits))) ++bad;
  }
  atomicAdd(&r[0], h);
  atomicAdd(&r[1], bad);
}
__global__ void hash_kernel(const uint64_t *k, uint64_t n, unsigned long long *r) {
  unsigned long long h = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    h += nut::mix64(k[i]);
  atomicAdd(&r[0], h);
}

__global__ void copy_kernel(const uint64_t *__restrict__ a, uint64_t *__restrict__ b, uint64_t n) {
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2; i < n; i += (uint64_t)gridDim.x * blockDim.x * 2)
    __builtin_nontemporal_store(__builtin_nontemporal_load((const nut::u64x2 *)(a + i)), (nut::u64x2 *)(b + i));
}

// one exact scatter level of keys by their top BITS bits; persistent, tiles of T x ITEMS keys
template <int BITS, int T, int ITEMS>
__global__ __launch_bounds__(T) void bins_scatter(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                  uint64_t n, unsigned long long *__restrict__ cursor) {
  constexpr int B = 1 << BITS, W = T / 64, PER = B >= T ? B / T : 1;
  constexpr uint32_t TILE = T * ITEMS;
  static_assert(TILE < (1u << (32 - BITS)), "rank bits");
  __shared__ uint64_t s_stage[TILE];
  __shared__ uint16_t s_dig[TILE];
  __shared__ uint32_t s_cnt[B], s_tex[B];
  __shared__ uint64_t s_gb[B];
  __shared__ uint32_t s_wsum[W];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t ntiles = (n + TILE - 1) / TILE;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t lo = tile * TILE;
    const uint32_t cnt = n - lo < TILE ? (uint32_t)(n - lo) : TILE;
    for (int i = tid; i < B; i += T) s_cnt[i] = 0;
    __syncthreads();
    uint64_t k[ITEMS];
    uint32_t sd[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) k[i] = __builtin_nontemporal_load(in + lo + ((uint32_t)(i * T + tid) < cnt ? (uint32_t)(i * T + tid) : cnt - 1));
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t d = (uint32_t)(k[i] >> (64 - BITS));
      const uint32_t r = (uint32_t)(i * T + tid) < cnt ? atomicAdd(&s_cnt[d], 1u) : 0u;
      sd[i] = d | (r << BITS);
    }
    __syncthreads();
    uint32_t loc[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int b = tid * PER + j;
      loc[j] = b < B ? s_cnt[b] : 0u;
      sum += loc[j];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (int w = 0; w < wave; ++w) run += s_wsum[w];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int b = tid * PER + j;
      if (b < B) {
        s_tex[b] = run;
        const uint64_t gb = loc[j] ? (uint64_t)atomicAdd(&cursor[b], (unsigned long long)loc[j]) : 0;
        s_gb[b] = gb - run;
        run += loc[j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t d = sd[i] & (B - 1);
      const uint32_t slot = (sd[i] >> BITS) + s_tex[d];
      if ((uint32_t)(i * T + tid) < cnt) {
        s_stage[slot] = k[i];
        s_dig[slot] = (uint16_t)d;
      }
    }
    __syncthreads();
    for (uint32_t j = tid; j < cnt; j += T) __builtin_nontemporal_store(s_stage[j], out + s_gb[s_dig[j]] + j);
    __syncthreads();
  }
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

template <int BITS, int T, int ITEMS>
static void run(const uint64_t *in, uint64_t *out, uint64_t n, unsigned long long *cur, unsigned long long *chk,
                unsigned long long want, int ncu, const char *name) {
  constexpr int B = 1 << BITS;
  auto kern = bins_scatter<BITS, T, ITEMS>;
  CK(hipMemset(cur, 0, B * 8));
  hipLaunchKernelGGL(hist_kernel<BITS>, dim3(1024), dim3(256), 0, 0, in, n, cur);
  std::vector<unsigned long long> h(B), c0(B);
  CK(hipMemcpy(h.data(), cur, B * 8, hipMemcpyDeviceToHost));
  unsigned long long a = 0;
  for (int d = 0; d < B; ++d) c0[d] = a, a += h[d];
  int per_cu = 1;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, T, 0));
  const unsigned grid = (unsigned)std::max(1, ncu * per_cu);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e9;
  for (int r = 0; r < 3; ++r) {
    CK(hipMemcpy(cur, c0.data(), B * 8, hipMemcpyHostToDevice));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(T), 0, 0, in, out, n, cur);
    CK(hipEventRecord(e1));
    best = std::min(best, elapsed(e0, e1));
  }
  CK(hipGetLastError());
  unsigned long long res[2] = {0, 0};
  CK(hipMemset(chk, 0, 16));
  hipLaunchKernelGGL(check_kernel, dim3(4096), dim3(256), 0, 0, out, n, BITS, chk);
  CK(hipMemcpy(res, chk, 16, hipMemcpyDeviceToHost));
  printf("%-30s %4d bins  %2d WG/CU: %7.3f ms  %6.0f GB/s  keys/run/tile %6.1f  %s\n", name, B, per_cu, best,
         16.0 * n / best / 1e6, (double)(T * ITEMS) / B,
         res[0] == want && res[1] == 0 ? "permutation ok, digits ordered" : "WRONG");
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? (uint64_t)atof(argv[1]) : 1250000000ull;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  uint64_t *in, *out;
  unsigned long long *cur, *chk;
  CK(hipMalloc(&in, n * 8));
  CK(hipMalloc(&out, n * 8 + 256));
  CK(hipMalloc(&cur, 4096 * 8));
  CK(hipMalloc(&chk, 16));
  hipLaunchKernelGGL(gen_keys, dim3(8192), dim3(256), 0, 0, in, n);
  CK(hipMemset(chk, 0, 16));
  hipLaunchKernelGGL(hash_kernel, dim3(4096), dim3(256), 0, 0, in, n, chk);
  unsigned long long want = 0;
  CK(hipMemcpy(&want, chk, 8, hipMemcpyDeviceToHost));
  {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(copy_kernel, dim3(8192), dim3(256), 0, 0, in, out, n);
      CK(hipEventRecord(e1));
      best = std::min(best, elapsed(e0, e1));
    }
    printf("%-30s                   %7.3f ms  %6.0f GB/s\n", "copy of the keys", best, 16.0 * n / best / 1e6);
  }
  printf("keys %llu (uniform 64-bit), exact layout, digit = top bits\n", (unsigned long long)n);
  run<3, 512, 16>(in, out, n, cur, chk, want, ncu, "P = 8 partition (512 x 16)");
  run<9, 512, 16>(in, out, n, cur, chk, want, ncu, "level 0, 512 bins (512 x 16)");
  run<9, 1024, 14>(in, out, n, cur, chk, want, ncu, "level 0, 512 bins (1024 x 14)");
  run<10, 512, 16>(in, out, n, cur, chk, want, ncu, "fold at P = 2 (512 x 16)");
  run<12, 512, 16>(in, out, n, cur, chk, want, ncu, "fold at P = 8 (512 x 16)");
  run<12, 1024, 8>(in, out, n, cur, chk, want, ncu, "fold at P = 8 (1024 x 8)");
  run<3, 512, 16>(in, out, n, cur, chk, want, ncu, "P = 8 partition again");
  run<12, 512, 16>(in, out, n, cur, chk, want, ncu, "fold at P = 8 again");
  return 0;
}
