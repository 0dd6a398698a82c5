// gp_tune.hip — variant sweep of the partitioned group-by's scatter (not product code; the
// product kernel is nutdb_amd/csrc/gpart.hpp gp_scatter_kernel, included here).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include scripts/tune/gp_tune.hip -o scripts/tune/bin/gp_tune
// run:   gp_tune [rows] [groups]   (1e9 records of the config-3 pool keys + dyadic values, G = 1e5)
// One level-0 pass in the optimistic layout (digit d owns rows [d * cap, (d + 1) * cap)),
// best of 3 per variant; the product variant is checked: every record lands in its digit's
// region and the (key, value) multiset is unchanged.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "../../nutdb_amd/csrc/gpart.hpp"

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                                      \
    }                                                               \
  } while (0)

__global__ void gen_kv(uint64_t *k, uint64_t *v, uint64_t n, uint64_t groups) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    k[i] = nut::mix64((nut::gen_u64(0x51, i) % groups) ^ nut::kPoolSalt);
    const double d = (double)(nut::gen_u64(0x52, i) >> 44) / 64.0;
    v[i] = (uint64_t)__double_as_longlong(d);
  }
}

// sum of mix64(k ^ mix64(v)) over records, and the records outside their digit's region
__global__ void check_kv(const uint64_t *k, const uint64_t *v, const unsigned long long *cur, uint64_t cap,
                         int bits, unsigned long long *out) {
  unsigned long long h = 0, bad = 0, cnt = 0;
  for (uint32_t d = blockIdx.x; d < (1u << bits); d += gridDim.x) {
    const uint64_t a = (uint64_t)d * cap, b = cur[d];
    for (uint64_t i = a + threadIdx.x; i < b; i += blockDim.x) {
      h += nut::mix64(k[i] ^ nut::mix64(v[i]));
      bad += (nut::owner_hash(k[i], 0, 1) >> (64 - bits)) != d;
      ++cnt;
    }
  }
  atomicAdd(&out[0], h);
  atomicAdd(&out[1], bad);
  atomicAdd(&out[2], cnt);
}
__global__ void hash_src(const uint64_t *k, const uint64_t *v, uint64_t n, unsigned long long *out) {
  unsigned long long h = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    h += nut::mix64(k[i] ^ nut::mix64(v[i]));
  atomicAdd(&out[0], h);
}

__global__ void copy2(const uint64_t *__restrict__ a, const uint64_t *__restrict__ b, uint64_t *__restrict__ c,
                      uint64_t *__restrict__ d, uint64_t n) {
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2; i < n; i += (uint64_t)gridDim.x * blockDim.x * 2) {
    *(nut::u64x2 *)(c + i) = __builtin_nontemporal_load((const nut::u64x2 *)(a + i));
    *(nut::u64x2 *)(d + i) = __builtin_nontemporal_load((const nut::u64x2 *)(b + i));
  }
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms;
  CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

struct Ctx {
  uint64_t n, rows;
  uint64_t *k, *v, *dk, *dv;
  nut::GpSeg *dseg;
  uint32_t *dts;
  uint32_t nst;
  unsigned long long *cur, *chk;
  unsigned long long want;
  hipEvent_t e0, e1;
  int ncu;
};

template <int T, int VAR, int BITS = 8>
static void run(Ctx &c, const char *name, bool check) {
  auto kern = nut::gp_scatter_kernel<1, T, VAR, BITS>;
  constexpr int BINS = 1 << BITS;
  const uint64_t cap = ((2 * c.rows - 2 * nut::GP_TILE) / BINS) & ~1ull;
  std::vector<unsigned long long> cur0(BINS + 1, 0);
  for (int d = 0; d < BINS; ++d) cur0[d] = (uint64_t)d * cap;
  nut::GpSeg seg{0, c.n, 0, 0};
  seg.ocap = cap;
  CK(hipMemcpy(c.dseg, &seg, sizeof seg, hipMemcpyHostToDevice));
  int per_cu = 1;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, T, 0));
  constexpr uint32_t TILE = T * nut::GP_ITEMS;
  // tiles of the one segment
  const uint32_t nst = (uint32_t)((c.n + 2 * TILE - 1) / (2 * TILE)) * 2;  // (2 * GP_TILE tiles in the product)
  (void)nst;
  const uint32_t ntiles = (uint32_t)((c.n + TILE - 1) / TILE);
  std::vector<uint32_t> ts(ntiles, 0);
  uint32_t *dts;
  CK(hipMalloc(&dts, ntiles * 4));
  CK(hipMemcpy(dts, ts.data(), ntiles * 4, hipMemcpyHostToDevice));
  const unsigned grid = (unsigned)std::min<uint64_t>(ntiles, (uint64_t)c.ncu * per_cu);
  nut::GpArrays ar{};
  ar.src[1] = c.k;
  ar.src[3] = c.v;
  ar.dst[1] = c.dk;
  ar.dst[3] = c.dv;
  ar.narr = 4;
  float best = 1e9;
  for (int r = 0; r < 3; ++r) {
    CK(hipMemcpy(c.cur, cur0.data(), cur0.size() * 8, hipMemcpyHostToDevice));
    CK(hipEventRecord(c.e0));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(T), 0, 0, ar, (const nut::GpSeg *)c.dseg, (const uint32_t *)dts, ntiles,
                       64 - BITS, 0, c.cur, 0ull, (uint64_t)BINS * cap, c.cur + BINS, nut::GpRange{},
                       (unsigned long long *)nullptr, (uint64_t)0, (unsigned long long *)nullptr);
    CK(hipEventRecord(c.e1));
    best = std::min(best, elapsed(c.e0, c.e1));
  }
  CK(hipGetLastError());
  char res[128] = "-";
  if (check) {
    unsigned long long h[3] = {0, 0, 0}, over = 0;
    CK(hipMemcpy(&over, c.cur + BINS, 8, hipMemcpyDeviceToHost));
    CK(hipMemset(c.chk, 0, 24));
    hipLaunchKernelGGL(check_kv, dim3(256), dim3(256), 0, 0, c.dk, c.dv, c.cur, cap, BITS, c.chk);
    CK(hipMemcpy(h, c.chk, 24, hipMemcpyDeviceToHost));
    snprintf(res, sizeof res, "records %llu/%llu misplaced %llu multiset %s overflow %llu", h[2],
             (unsigned long long)c.n, h[1], h[0] == c.want ? "ok" : "DIFFERS", over);
  }
  printf("%-34s %d WG/CU grid %5u: %7.3f ms  %6.0f GB/s  %s\n", name, per_cu, grid, best, 32.0 * c.n / best / 1e6, res);
  CK(hipFree(dts));
}

int main(int argc, char **argv) {
  Ctx c;
  c.n = argc > 1 ? (uint64_t)atof(argv[1]) : 1000000000ull;
  const uint64_t groups = argc > 2 ? (uint64_t)atof(argv[2]) : 100000ull;
  CK(hipDeviceGetAttribute(&c.ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t rows = (c.n + 2 * 65536 + 64 + 31) & ~31ull;
  c.rows = rows;
  CK(hipMalloc(&c.k, c.n * 8));
  CK(hipMalloc(&c.v, c.n * 8));
  CK(hipMalloc(&c.dk, 2 * rows * 8 + (1 << 20)));
  CK(hipMalloc(&c.dv, 2 * rows * 8 + (1 << 20)));
  CK(hipMalloc(&c.cur, (1024 + 1) * 8));
  CK(hipMalloc(&c.chk, 32));
  CK(hipMalloc(&c.dseg, sizeof(nut::GpSeg)));
  CK(hipEventCreate(&c.e0));
  CK(hipEventCreate(&c.e1));
  hipLaunchKernelGGL(gen_kv, dim3(8192), dim3(256), 0, 0, c.k, c.v, c.n, groups);
  CK(hipMemset(c.chk, 0, 8));
  hipLaunchKernelGGL(hash_src, dim3(4096), dim3(256), 0, 0, c.k, c.v, c.n, c.chk);
  CK(hipMemcpy(&c.want, c.chk, 8, hipMemcpyDeviceToHost));
  {
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(c.e0));
      hipLaunchKernelGGL(copy2, dim3(8192), dim3(256), 0, 0, c.k, c.v, c.dk, c.dv, c.n);
      CK(hipEventRecord(c.e1));
      best = std::min(best, elapsed(c.e0, c.e1));
    }
    printf("%-34s                   %7.3f ms  %6.0f GB/s\n", "copy 2 arrays (HBM floor)", best, 32.0 * c.n / best / 1e6);
  }
  printf("records %llu, groups %llu\n", (unsigned long long)c.n, (unsigned long long)groups);
  if (argc > 3 && std::string(argv[3]) == "layout") {
    // the product's output layout (aggregate.hip groupby_partitioned_direct: every array's
    // regions in one gp_data allocation, array k at row k * 2 * rows) vs one allocation per
    // array, interleaved on one box
    uint64_t *joint = nullptr, *sep_k = c.dk, *sep_v = c.dv;
    CK(hipMalloc(&joint, 4 * rows * 8 + 256));
    for (int r = 0; r < 2; ++r) {
      c.dk = sep_k, c.dv = sep_v;
      run<1024, 1, 7>(c, "128 bins, separate allocations", true);
      c.dk = joint, c.dv = joint + 2 * rows;
      run<1024, 1, 7>(c, "128 bins, product layout (joint)", true);
    }
    return 0;
  }
  run<1024, 1>(c, "product <1,1024> (nt stores)", true);
  if (argc > 3) return 0;  // profiling runs: the product variant only
  run<1024, 1, 7>(c, "<1,1024> nt, 128 bins (G = 1e5)", true);
  run<1024, 33, 7>(c, "<1,1024> nt early loads, 128 bins", true);
  run<1024, 1, 7>(c, "<1,1024> nt, 128 bins again", true);
  run<1024, 33, 7>(c, "<1,1024> nt early loads again", true);
  run<512, 1, 7>(c, "<1,512> nt, 128 bins, 2 WG/CU", true);
  run<512, 1, 6>(c, "<1,512> nt, 64 bins, 2 WG/CU", true);
  run<1024, 17, 7>(c, "<1,1024> 128 bins private cursors", false);
  run<1024, 3, 7>(c, "<1,1024> 128 bins no stores", false);
  run<512, 3, 7>(c, "<1,512> 128 bins no stores", false);
  run<1024, 0>(c, "<1,1024> plain stores", true);
  run<1024, 4>(c, "<1,1024> tile-sequential out", false);
  run<1024, 2>(c, "<1,1024> no stores", false);
  run<1024, 8>(c, "<1,1024> lookups + sequential out", false);
  run<512, 0>(c, "<1,512>", true);
  run<1024, 0, 7>(c, "<1,1024> 128 bins", true);
  run<1024, 4, 7>(c, "<1,1024> 128 bins tile-sequential", false);
  run<1024, 0, 6>(c, "<1,1024> 64 bins", true);
  return 0;
}
