// local_tune.hip — variant sweep of the MSD sort's local-sort kernel (not product code; the
// product kernel is nutdb_amd/csrc/msd_sort.hip ms_local_kernel, included here).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/tune/local_tune.hip -o scripts/tune/bin/local_tune
// run:   local_tune [nseg] [seglen]   (262144 segments of 4768 keys = the 1.25e9-key sort's second level)
// Every segment's keys share their top 18 bits (as after two 9-bit levels); each variant is
// timed best-of-3 and checked: sorted inside every segment and the same multiset.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define NUT_MSD_KERNELS_ONLY
#ifndef LT_PLAIN  // -DLT_PLAIN: the product kernel as built (no stop checks, no cycle stamps)
#define NUT_MSD_PROFILE_STOP
#define NUT_MSD_STAMPS
#endif
#include "../../nutdb_amd/csrc/msd_sort.hip"

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                                      \
    }                                                               \
  } while (0)

__global__ void gen_segs(uint64_t *c, uint64_t n, uint32_t seglen) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c[i] = ((i / seglen) << 46) | (nut::gen_u64(0x50, i) & ((1ull << 46) - 1));
}

__global__ void check(const uint64_t *d, uint64_t n, uint32_t seglen, unsigned long long *out) {
  unsigned long long bad = 0, h = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if ((i + 1) % seglen != 0 && i + 1 < n && d[i] > d[i + 1]) ++bad;
    h += nut::mix64(d[i]);
  }
  atomicAdd(&out[0], bad);
  atomicAdd(&out[1], h);
}

// copy of the same bytes (read segments, write them back): the HBM floor of the kernel
__global__ void copy_kernel(const uint64_t *__restrict__ s, uint64_t *__restrict__ d, uint64_t n) {
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2; i < n; i += (uint64_t)gridDim.x * blockDim.x * 2) {
    const nut::u64x2 v = __builtin_nontemporal_load((const nut::u64x2 *)(s + i));
    *(nut::u64x2 *)(d + i) = v;
  }
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms;
  CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

struct Ctx {
  uint64_t *src, *dst;
  uint64_t n;
  uint32_t seglen, nseg;
  nut::MsSeg *dseg;
  uint32_t *fb;
  unsigned long long *chk;
  unsigned long long want_hash;
  hipEvent_t e0, e1;
};

template <int T, int K, int SB, int WS, bool PF = true, int LK = 0>
static void run(Ctx &c, const char *name, int stop = 0) {
  auto kern = nut::ms_local_kernel<T, K, PF, SB, WS, LK>;
  int per_cu = 1, ncu = 256;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, T, 0));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  // persistent with the next segment's keys prefetched, or one workgroup per segment
  const unsigned grid = PF ? (unsigned)std::min<uint64_t>(c.nseg, (uint64_t)ncu * per_cu) : c.nseg;
#ifndef LT_PLAIN
  CK(hipMemcpyToSymbol(HIP_SYMBOL(nut::g_ms_stop), &stop, sizeof(int)));
#else
  if (stop) return;
#endif
  nut::MsBufs bf{nullptr, c.dst, c.src, nullptr};
  float best = 1e9;
  unsigned long long st[8] = {0};
  for (int r = 0; r < 3; ++r) {
    CK(hipMemset(c.fb, 0, 4));
#ifndef LT_PLAIN
    CK(hipMemcpyToSymbol(HIP_SYMBOL(nut::g_ms_stamp), st, sizeof(st)));
#endif
    CK(hipEventRecord(c.e0));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(T), 0, 0, bf, (const nut::MsSeg *)c.dseg, c.nseg, 0ull, c.fb);
    CK(hipEventRecord(c.e1));
    best = std::min(best, elapsed(c.e0, c.e1));
  }
#ifndef LT_PLAIN
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(nut::g_ms_stamp), sizeof(st)));
  if (!stop) {
    printf("   cycles per segment (thread 0 of each workgroup):");
    const char *ph[7] = {"ranks", "scan+windows", "place", "sort", "copy", "next", "-"};
    for (int k = 0; k < 6; ++k) printf(" %s %.0f", ph[k], (double)st[k] / c.nseg);
    printf("\n");
  }
#endif
  uint32_t nfb = 0;
  CK(hipMemcpy(&nfb, c.fb, 4, hipMemcpyDeviceToHost));
  unsigned long long h[2] = {0, 0};
  if (!stop) {
    CK(hipMemset(c.chk, 0, 16));
    hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, c.dst, c.n, c.seglen, c.chk);
    CK(hipMemcpy(h, c.chk, 16, hipMemcpyDeviceToHost));
  }
  printf("%-28s stop=%d %d WG/CU: %7.3f ms  %6.0f GB/s  unsorted %llu  multiset %s  fallback segs %u\n", name, stop,
         per_cu, best, 16.0 * c.n / best / 1e6, h[0], stop ? "-" : (h[1] == c.want_hash ? "ok" : "DIFFERS"), nfb);
}

int main(int argc, char **argv) {
  Ctx c;
  c.nseg = argc > 1 ? (uint32_t)atoi(argv[1]) : 262144u;
  c.seglen = argc > 2 ? (uint32_t)atoi(argv[2]) : 4768u;
  c.n = (uint64_t)c.nseg * c.seglen;
  CK(hipMalloc(&c.src, c.n * 8));
  CK(hipMalloc(&c.dst, c.n * 8));
  CK(hipMalloc(&c.chk, 16));
  CK(hipMalloc(&c.fb, (c.nseg + 1) * 4));
  std::vector<nut::MsSeg> segs(c.nseg);
  for (uint32_t i = 0; i < c.nseg; ++i) segs[i] = nut::MsSeg{(uint64_t)i * c.seglen, c.seglen, 2, 46};
  CK(hipMalloc(&c.dseg, c.nseg * sizeof(nut::MsSeg)));
  CK(hipMemcpy(c.dseg, segs.data(), c.nseg * sizeof(nut::MsSeg), hipMemcpyHostToDevice));
  CK(hipEventCreate(&c.e0));
  CK(hipEventCreate(&c.e1));
  hipLaunchKernelGGL(gen_segs, dim3(8192), dim3(256), 0, 0, c.src, c.n, c.seglen);
  CK(hipMemset(c.chk, 0, 16));
  hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, c.src, c.n, c.seglen, c.chk);
  unsigned long long h[2];
  CK(hipMemcpy(h, c.chk, 16, hipMemcpyDeviceToHost));
  c.want_hash = h[1];
  {
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(c.e0));
      hipLaunchKernelGGL(copy_kernel, dim3(8192), dim3(256), 0, 0, c.src, c.dst, c.n);
      CK(hipEventRecord(c.e1));
      best = std::min(best, elapsed(c.e0, c.e1));
    }
    printf("%-28s                 %7.3f ms  %6.0f GB/s\n", "copy (HBM floor)", best, 16.0 * c.n / best / 1e6);
  }
  printf("segments %u x %u keys\n", c.nseg, c.seglen);
  run<nut::LS_M_THREADS, nut::LS_M_ITEMS, 0, 0, false>(c, "product M class 1 WG/segment");
  if (argc > 3) return 0;  // profiling runs: the product variant only
  run<256, 20, 11, 10, false>(c, "round-5 <256,20> SB11 WS10");
  run<512, 10, 11, 10, false>(c, "<512,10> SB11 WS10 1 WG/seg");
  run<1024, 5, 11, 10, false>(c, "<1024,5> SB11 WS10 1 WG/seg");
  run<256, 20, 11, 10, false, 3072>(c, "<256,20> SB11 WS10 LK3072");
  return 0;
  run<512, 12, 0, 0>(c, "default: load only", 1);
  run<512, 12, 0, 0>(c, "default: + ranks/stage", 3);
  run<512, 12, 0, 0>(c, "default: + windows", 4);
  return 0;
}
