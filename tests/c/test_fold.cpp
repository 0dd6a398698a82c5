// CPU test of fold_sorted_groups (nutdb_amd/csrc/fold.hpp): random key-sorted results and
// random sorted extra groups (some keys present, some new), checked against a std::map
// merge — including sizes that take the threaded block moves.  Built and run by
// tests/test_fold_cpu.py.
#include <stdio.h>

#include <map>
#include <random>
#include <vector>

#include "fold.hpp"

using namespace nut::fold;

static int check(uint64_t n, uint64_t m, double fresh_frac, uint64_t seed, int na) {
  std::mt19937_64 rng(seed);
  const int32_t kinds[4] = {kSumF64, 2 /* COUNT */, kMinI64, kMaxI64};
  std::vector<int64_t> base;
  for (uint64_t i = 0; i < n; ++i) base.push_back((int64_t)(rng() >> 1) - (int64_t)(1ull << 61));
  std::sort(base.begin(), base.end());
  base.erase(std::unique(base.begin(), base.end()), base.end());
  n = base.size();
  std::map<int64_t, std::vector<uint64_t>> want;
  const uint64_t cap = n + m + 8;
  std::vector<int64_t> keys(cap);
  std::vector<uint64_t> aggs(cap * na);
  for (uint64_t i = 0; i < n; ++i) {
    keys[i] = base[i];
    std::vector<uint64_t> w(na);
    for (int a = 0; a < na; ++a) {
      if (kinds[a] == kSumF64) { double d = (double)(rng() % 1000) / 8; memcpy(&w[a], &d, 8); }
      else w[a] = rng() % 100000;
    }
    for (int a = 0; a < na; ++a) aggs[i * na + a] = w[a];
    want[base[i]] = w;
  }
  std::vector<int64_t> extra;
  for (uint64_t j = 0; j < m; ++j) {
    const bool fresh = (double)(rng() % 1000000) / 1e6 < fresh_frac || n == 0;
    extra.push_back(fresh ? (int64_t)(rng() >> 1) - (int64_t)(1ull << 61) : base[rng() % n]);
  }
  std::sort(extra.begin(), extra.end());
  extra.erase(std::unique(extra.begin(), extra.end()), extra.end());
  std::vector<uint64_t> hw;
  for (int64_t k : extra) {
    std::vector<uint64_t> w(na);
    for (int a = 0; a < na; ++a) {
      if (kinds[a] == kSumF64) { double d = (double)(rng() % 1000) / 8; memcpy(&w[a], &d, 8); }
      else w[a] = rng() % 100000;
      hw.push_back(w[a]);
    }
    auto it = want.find(k);
    if (it == want.end()) { want[k] = w; continue; }
    for (int a = 0; a < na; ++a) {
      uint64_t &x = it->second[a];
      if (kinds[a] == kSumF64) { double dx, dy; memcpy(&dx, &x, 8); memcpy(&dy, &w[a], 8); dx += dy; memcpy(&x, &dx, 8); }
      else if (kinds[a] == kMinI64) x = std::min<int64_t>(x, w[a]);
      else if (kinds[a] == kMaxI64) x = std::max<int64_t>(x, w[a]);
      else x += w[a];
    }
  }
  bool over = false;
  const uint64_t got = fold_sorted_groups(keys.data(), aggs.data(), n, cap, extra, hw, kinds, na, &over);
  if (over || got != want.size()) { printf("FAIL count n=%llu m=%llu: %llu vs %zu\n", (unsigned long long)n, (unsigned long long)m, (unsigned long long)got, want.size()); return 1; }
  uint64_t i = 0;
  for (auto &kv : want) {
    if (keys[i] != kv.first) { printf("FAIL key at %llu\n", (unsigned long long)i); return 1; }
    for (int a = 0; a < na; ++a)
      if (aggs[i * na + a] != kv.second[a]) { printf("FAIL agg at %llu/%d\n", (unsigned long long)i, a); return 1; }
    ++i;
  }
  return 0;
}

int main() {
  int bad = 0;
  bad += check(0, 10, 1.0, 1, 2);         // empty result: every group fresh
  bad += check(1000, 0, 0.5, 2, 4);       // nothing to fold
  bad += check(1000, 300, 0.0, 3, 4);     // combines only
  bad += check(1000, 300, 1.0, 4, 1);     // fresh only
  bad += check(5000, 2000, 0.3, 5, 3);    // mixed, serial moves
  bad += check(3000000, 20000, 0.3, 6, 4);   // threaded moves
  bad += check(2000000, 7, 1.0, 7, 2);       // fewer fresh keys than threads
  bad += check(1500000, 300000, 0.9, 8, 4);  // many fresh keys
  printf(bad ? "FAILED %d\n" : "ok\n", bad);
  return bad != 0;
}
