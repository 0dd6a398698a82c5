// hk_tune.hip — timing variants of the ordered group-by's heavy-key pass (not product code;
// the product kernel is nutdb_amd/csrc/heavy.hpp hk_split_kernel, included here).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I nutdb_amd/csrc scripts/tune/hk_tune.hip -o scripts/tune/bin/hk_tune
// run:   hk_tune [rows] [pool]   (1e9 Zipf-like keys over a 1e7-key pool, one f64 value)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <unordered_map>
#include <vector>

#include "heavy.hpp"

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                                      \
    }                                                               \
  } while (0)

// the product's GEN_SKEW_KEY / dyadic-value generators (api.hip)
__global__ void gen(uint64_t *k, uint64_t *v, uint64_t n, uint64_t pool, int skew) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t u = nut::gen_u64(0x51, i);
    const uint64_t idx = skew ? ((u % pool) >> (((nut::mix64(u) >> 59) * 3) >> 2)) : u % pool;
    k[i] = nut::mix64(idx ^ nut::kPoolSalt);
    v[i] = nut::gen_u64(0x52, i);
  }
}
__global__ void copy2(const uint64_t *a, const uint64_t *b, uint64_t *c, uint64_t *d, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    c[i] = __builtin_nontemporal_load(a + i);
    d[i] = __builtin_nontemporal_load(b + i);
  }
}

struct Ctx {
  uint64_t n, *k, *v, *ok, *ov, *hk, *hagg, *cnt, s1, s2;
  uint16_t *slot;
  uint32_t h;
  int ncu;
  hipEvent_t e0, e1;
};

template <int VAR>
static void run(Ctx &c, const char *name, uint32_t h) {
  auto kern = nut::hk_split_kernel<1, VAR>;
  int per_cu = 1;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, nut::HK_THREADS, 0));
  const uint64_t ntiles = (c.n + nut::HK_TILE - 1) / nut::HK_TILE;
  const uint64_t grid = std::min<uint64_t>(ntiles, (uint64_t)c.ncu * per_cu), chunk = (ntiles + grid - 1) / grid;
  nut::HkArgs a{};
  a.key = c.k;
  a.val[0] = c.v;
  a.okey = c.ok;
  a.oval[0] = c.ov;
  a.n = c.n;
  a.chunk = chunk;
  a.nv = 1;
  a.na = 1;
  a.kind[0] = nut::AK_SUM_F64;
  a.arg[0] = 0;
  a.hk = (const int64_t *)c.hk;
  a.slot = c.slot;
  a.seed1 = c.s1;
  a.seed2 = c.s2;
  a.h = h;
  a.hagg = c.hagg;
  a.count = c.cnt;
  float best = 1e9;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(c.e0));
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(nut::HK_THREADS), 0, 0, a);
    CK(hipEventRecord(c.e1));
    CK(hipEventSynchronize(c.e1));
    float ms;
    CK(hipEventElapsedTime(&ms, c.e0, c.e1));
    best = std::min(best, ms);
  }
  std::vector<uint64_t> cnt(grid);
  CK(hipMemcpy(cnt.data(), c.cnt, grid * 8, hipMemcpyDeviceToHost));
  uint64_t kept = 0;
  for (uint64_t x : cnt) kept += x;
  printf("%-34s %4d WG/CU  %7.3f ms  kept %.3f of %llu rows\n", name, per_cu, best, (double)kept / c.n,
         (unsigned long long)c.n);
}

int main(int argc, char **argv) {
  Ctx c;
  c.n = argc > 1 ? (uint64_t)atof(argv[1]) : 1000000000ull;
  const uint64_t pool = argc > 2 ? (uint64_t)atof(argv[2]) : 10000000ull;
  CK(hipDeviceGetAttribute(&c.ncu, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipMalloc(&c.k, c.n * 8));
  CK(hipMalloc(&c.v, c.n * 8));
  CK(hipMalloc(&c.ok, (c.n + (8ull << 20)) * 8));
  CK(hipMalloc(&c.ov, (c.n + (8ull << 20)) * 8));
  CK(hipMalloc(&c.hk, nut::HK_MAX * 8));
  CK(hipMalloc(&c.hagg, nut::HK_MAX * 8));
  CK(hipMalloc(&c.cnt, 65536 * 8));
  CK(hipMalloc(&c.slot, nut::HK_SLOTS * 2));
  CK(hipEventCreate(&c.e0));
  CK(hipEventCreate(&c.e1));
  for (int skew = 1; skew >= 0; --skew) {
    hipLaunchKernelGGL(gen, dim3(8192), dim3(256), 0, 0, c.k, c.v, c.n, pool, skew);
    // the heavy keys as the product picks them: strided 64 Ki sample, >= 4 hits, top 1024
    std::vector<uint64_t> smp(65536), all(c.n > 0 ? 1 : 0);
    std::unordered_map<uint64_t, uint32_t> cnt;
    for (uint32_t i = 0; i < 65536; ++i) {
      uint64_t x;
      CK(hipMemcpy(&x, c.k + (c.n / 65536) * i, 8, hipMemcpyDeviceToHost));
      ++cnt[x];
    }
    std::vector<std::pair<uint32_t, uint64_t>> cand;
    for (auto &kv : cnt)
      if (kv.second >= 3) cand.emplace_back(kv.second, kv.first);
    std::sort(cand.rbegin(), cand.rend());
    if (cand.size() > (size_t)nut::HK_MAX) cand.resize(nut::HK_MAX);
    std::vector<uint64_t> hk;
    for (auto &x : cand) hk.push_back(x.second);
    std::sort(hk.begin(), hk.end(), [](uint64_t a, uint64_t b) { return (int64_t)a < (int64_t)b; });
    c.h = (uint32_t)hk.size();
    if (c.h) CK(hipMemcpy(c.hk, hk.data(), c.h * 8, hipMemcpyHostToDevice));
    std::vector<uint16_t> slot(nut::HK_SLOTS);
    c.s1 = nut::mix64(0x9E3779B97F4A7C15ull);
    c.s2 = nut::mix64(0x9E3779B97F4A7C16ull);
    if (!nut::hk_cuckoo((const int64_t *)hk.data(), c.h, c.s1, c.s2, slot.data())) printf("cuckoo build failed\n");
    CK(hipMemcpy(c.slot, slot.data(), nut::HK_SLOTS * 2, hipMemcpyHostToDevice));
    printf("%s keys: %u heavy\n", skew ? "Zipf-like" : "uniform", c.h);
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(c.e0));
      hipLaunchKernelGGL(copy2, dim3(c.ncu * 8), dim3(256), 0, 0, c.k, c.v, c.ok, c.ov, c.n);
      CK(hipEventRecord(c.e1));
      CK(hipEventSynchronize(c.e1));
      float ms;
      CK(hipEventElapsedTime(&ms, c.e0, c.e1));
      best = std::min(best, ms);
    }
    printf("%-34s          %7.3f ms  (read + write all rows)\n", "copy 2 arrays", best);
    run<0>(c, "product", c.h);
    run<0>(c, "product, no heavy keys", 0);
    run<1>(c, "no lookups", c.h);
    run<2>(c, "no accumulator atomics", c.h);
    run<4>(c, "no stores", c.h);
    run<6>(c, "lookups only", c.h);
    run<7>(c, "loads + scan only", c.h);
  }
  return 0;
}
