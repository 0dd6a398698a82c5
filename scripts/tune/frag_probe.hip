// frag_probe.hip — does the placement of a large random-read table change its read rate?
// (not part of the product: the r05 join cliff).  The hash join reads an
// 8 GB slot table at random; a table whose pages map with small fragments would miss the
// GPU TLB on nearly every read.  This times random 16-B reads (the probe's access) over an
// 8 GB buffer that is
//   fresh   — hipMalloc on an unfragmented device,
//   frag    — hipMalloc after most of HBM was filled with 2 MB + 4 KB buffers and every
//             other one freed (free memory only in odd-sized holes),
//   vmm     — hipMemCreate handles of the recommended granularity mapped into one range,
//             in the same fragmented state.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/tune/frag_probe.hip -o scripts/tune/bin/frag_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../../nutdb_amd/csrc/common.hpp"

using namespace nut;

__global__ __launch_bounds__(256) void rr16_kernel(const uint64_t *__restrict__ a, uint64_t mask, uint64_t n,
                                                   uint64_t seed, uint64_t *__restrict__ out) {
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t acc = 0;
  for (uint64_t base = lane * 8; base < n; base += stride * 8) {
    uint64_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t idx = (mix64(base + k + seed) & mask) & ~1ull;
      const ulonglong2 x = *(const ulonglong2 *)(a + idx);
      v[k] = x.x ^ x.y;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= v[k];
  }
  out[lane] = acc;
}

static double rate(const uint64_t *a, uint64_t words, uint64_t *out, int grid) {
  const uint64_t n = 1ull << 28;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(rr16_kernel, dim3(grid), dim3(256), 0, 0, a, words - 1, n, 1, out);
  (void)hipEventRecord(e0);
  const int R = 5;
  for (int r = 0; r < R; ++r) hipLaunchKernelGGL(rr16_kernel, dim3(grid), dim3(256), 0, 0, a, words - 1, n, r + 2, out);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return n * (double)R / (ms * 1e-3) / 1e9;
}

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

int main(int argc, char **argv) {
  const double fill_frac = argc > 1 ? atof(argv[1]) : 0.8;  // of free HBM filled before the holes
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = cus * 16;
  uint64_t *out = nullptr;
  CK(hipMalloc(&out, (size_t)grid * 256 * 8));
  const size_t tbl = 8ull << 30;
  const uint64_t words = tbl / 8;
  {
    uint64_t *a = nullptr;
    CK(hipMalloc(&a, tbl));
    CK(hipMemset(a, 1, tbl));
    printf("fresh   hipMalloc 8 GB: %.1f G random 16-B reads/s\n", rate(a, words, out, grid));
    CK(hipFree(a));
  }
  // fragment: fill, then free every other buffer
  size_t fr = 0, total = 0;
  CK(hipMemGetInfo(&fr, &total));
  const size_t piece = (2ull << 20) + 4096;
  const size_t npieces = (size_t)(fr * fill_frac) / piece;
  std::vector<void *> pieces(npieces, nullptr);
  size_t got = 0;
  for (size_t i = 0; i < npieces; ++i) {
    if (hipMalloc(&pieces[i], piece) != hipSuccess) {
      (void)hipGetLastError();
      pieces[i] = nullptr;
      break;
    }
    ++got;
  }
  for (size_t i = 0; i < got; i += 2) {
    (void)hipFree(pieces[i]);
    pieces[i] = nullptr;
  }
  CK(hipMemGetInfo(&fr, &total));
  printf("fragmented: %zu pieces of %zu B, every other freed; free %.1f GB of %.1f GB\n", got, piece, fr / 1e9,
         total / 1e9);
  {
    uint64_t *a = nullptr;
    CK(hipMalloc(&a, tbl));
    CK(hipMemset(a, 1, tbl));
    printf("frag    hipMalloc 8 GB: %.1f G random 16-B reads/s\n", rate(a, words, out, grid));
    CK(hipFree(a));
  }
  {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0, rec = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    CK(hipMemGetAllocationGranularity(&rec, &prop, hipMemAllocationGranularityRecommended));
    printf("vmm granularity: minimum %zu, recommended %zu\n", gran, rec);
    const size_t g = std::max<size_t>(rec, 2ull << 20);
    void *va = nullptr;
    CK(hipMemAddressReserve(&va, tbl, g, nullptr, 0));
    std::vector<hipMemGenericAllocationHandle_t> hs;
    const size_t chunk = 256ull << 20;  // 256 MB handles
    for (size_t off = 0; off < tbl; off += chunk) {
      hipMemGenericAllocationHandle_t h;
      CK(hipMemCreate(&h, chunk, &prop, 0));
      CK(hipMemMap((char *)va + off, chunk, 0, h, 0));
      hs.push_back(h);
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(va, tbl, &acc, 1));
    CK(hipMemset(va, 1, tbl));
    printf("vmm     8 GB in 256 MB handles: %.1f G random 16-B reads/s\n", rate((const uint64_t *)va, words, out, grid));
    CK(hipMemUnmap(va, tbl));
    for (auto h : hs) CK(hipMemRelease(h));
    CK(hipMemAddressFree(va, tbl));
  }
  for (void *p : pieces)
    if (p) (void)hipFree(p);
  {
    uint64_t *a = nullptr;
    CK(hipMalloc(&a, tbl));
    CK(hipMemset(a, 1, tbl));
    printf("after   hipMalloc 8 GB: %.1f G random 16-B reads/s\n", rate(a, words, out, grid));
    CK(hipFree(a));
  }
  CK(hipFree(out));
  return 0;
}
