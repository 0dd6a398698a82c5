// randread.hip — random-read rate of the memory hierarchy at table sizes from L2 to HBM
// (not part of the product: it sizes the hash join's probe design).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/tune/randread.hip -o /tmp/randread
// Each lane issues K independent loads of W bytes at hashed offsets; prints G accesses/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../nutdb_amd/csrc/common.hpp"

using namespace nut;

template <int W, int K>
__global__ __launch_bounds__(256) void rr_kernel(const uint64_t *__restrict__ a, uint64_t mask, uint64_t n,
                                                 uint64_t seed, uint64_t *__restrict__ out) {
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t acc = 0;
  for (uint64_t base = lane * K; base < n; base += stride * K) {
    uint64_t v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t idx = (mix64(base + k + seed) & mask) & ~(uint64_t)(W / 8 - 1);
      if constexpr (W == 16) {
        const ulonglong2 x = *(const ulonglong2 *)(a + idx);
        v[k] = x.x ^ x.y;
      } else {
        v[k] = a[idx];
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) acc ^= v[k];
  }
  out[lane] = acc;
}

template <int W, int K>
double run(const uint64_t *a, uint64_t words, uint64_t n, uint64_t *out, int grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((rr_kernel<W, K>), dim3(grid), dim3(256), 0, 0, a, words - 1, n, 1, out);
  hipEventRecord(e0);
  const int R = 5;
  for (int r = 0; r < R; ++r) hipLaunchKernelGGL((rr_kernel<W, K>), dim3(grid), dim3(256), 0, 0, a, words - 1, n, r + 2, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return n * (double)R / (ms * 1e-3) / 1e9;
}

int main() {
  int dev = 0, cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t max_bytes = 8ull << 30;
  uint64_t *a = nullptr, *out = nullptr;
  if (hipMalloc(&a, max_bytes) != hipSuccess) return 1;
  hipMemset(a, 1, max_bytes);
  const int grid = cus * 16;
  hipMalloc(&out, (size_t)grid * 256 * 8);
  const uint64_t n = 1ull << 28;  // accesses per launch
  printf("bytes        W=8,K=8   W=16,K=8  W=8,K=16  (G accesses/s)\n");
  for (uint64_t bytes : {4ull << 20, 16ull << 20, 64ull << 20, 128ull << 20, 256ull << 20, 512ull << 20, 2ull << 30,
                         8ull << 30}) {
    const uint64_t words = bytes / 8;
    const double r8 = run<8, 8>(a, words, n, out, grid), r16 = run<16, 8>(a, words, n, out, grid),
                 r8k = run<8, 16>(a, words, n, out, grid);
    printf("%10llu  %8.1f  %8.1f  %8.1f\n", (unsigned long long)bytes, r8, r16, r8k);
  }
  hipFree(a);
  hipFree(out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
