// fold.hpp — host-side merge of extra groups into a key-sorted group result
// (aggregate.hip groupby_ordered: the overflow arenas' groups and heavy keys that joined no
// partition).  Host C++ only, so the CPU tests compile it with g++ (tests/c/test_fold.cpp).
#pragma once
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

namespace nut {
namespace fold {

// aggregate kinds of the result words (the tables' AggKind values; aggregate.hip checks)
constexpr int kSumF64 = 0, kMinF64 = 3, kMaxF64 = 4, kMinI64 = 5, kMaxI64 = 6;
constexpr int kFoldThreads = 8;  // host threads of the block moves

// Fold groups sorted by key (hk, hw: result words, SELECT order) into a sorted host result
// of n groups with room for cap: equal keys combine by kind (SUM f64 adds, SUM i64 / COUNT
// wrap-add, MIN / MAX of f64 in the tables' total order: -0 < +0, NaN above +inf), the rest
// are merged in by one backward pass of block moves.  Returns the new count; *over when it
// exceeds cap (the caller then fails the call: equal keys may already be combined).
inline uint64_t fold_sorted_groups(int64_t *keys, uint64_t *aggs, uint64_t n, uint64_t cap,
                                   const std::vector<int64_t> &hk, const std::vector<uint64_t> &hw,
                                   const int32_t *kinds, int na, bool *over) {
  const uint64_t m = hk.size();
  auto ord = [](uint64_t b) { return (b >> 63) ? ~b : (b | 0x8000000000000000ull); };
  auto combine = [&](uint64_t *dst, const uint64_t *src) {
    for (int a = 0; a < na; ++a) {
      uint64_t &x = dst[a];
      const uint64_t y = src[a];
      switch (kinds[a]) {
        case kSumF64: {
          double dx, dy;
          memcpy(&dx, &x, 8);
          memcpy(&dy, &y, 8);
          dx += dy;
          memcpy(&x, &dx, 8);
          break;
        }
        case kMinF64: x = ord(y) < ord(x) ? y : x; break;
        case kMaxF64: x = ord(y) > ord(x) ? y : x; break;
        case kMinI64: x = (int64_t)y < (int64_t)x ? y : x; break;
        case kMaxI64: x = (int64_t)y > (int64_t)x ? y : x; break;
        default: x += y; break;  // SUM i64, COUNT
      }
    }
  };
  // each incoming key's place (hk ascending: a galloping search from the previous place, so
  // dense and sparse folds both stay near linear), equal keys combined in place; only the
  // keys not in the result yet move anything
  std::vector<uint64_t> pos;
  std::vector<uint32_t> fresh_j;
  uint64_t lo = 0;
  for (uint64_t j = 0; j < m; ++j) {
    uint64_t step = 1;
    while (lo + step < n && keys[lo + step] < hk[j]) step *= 2;
    lo = (uint64_t)(std::lower_bound(keys + lo + step / 2, keys + std::min(n, lo + step + 1), hk[j]) - keys);
    if (lo < n && keys[lo] == hk[j]) {
      combine(aggs + lo * na, &hw[j * na]);
    } else {
      fresh_j.push_back((uint32_t)j);
      pos.push_back(lo);
    }
  }
  const uint64_t fresh = fresh_j.size();
  if (n + fresh > cap) {
    *over = true;
    return n + fresh;
  }
  // backward: the block [p, end) of the rows after fresh key r's place moves up by the r + 1
  // fresh keys at or before it, then the key goes in front of it.  Old row i moves by the
  // count of fresh places <= i, so a fresh key near the front moves the whole result: the
  // blocks go to up to kFoldThreads threads, each a run of consecutive fresh keys and the
  // rows between them.  Group g's moves write over the first r0[g] rows of the next
  // groups' ranges, so every group first saves those head rows (joined before any move)
  // and takes them from the copy.
  auto move_rows = [&](uint64_t from, uint64_t to, uint64_t cnt) {
    memmove(keys + to, keys + from, cnt * 8);
    memmove(aggs + to * na, aggs + from * na, cnt * 8 * (size_t)na);
  };
  const int T = (int)std::min<uint64_t>(fresh, n >= (1ull << 20) ? kFoldThreads : 1);
  std::vector<uint64_t> r0(T + 1);
  for (int g = 0; g <= T; ++g) r0[g] = fresh * (uint64_t)g / (uint64_t)std::max(T, 1);
  auto start_of = [&](int g) { return g < T ? pos[r0[g]] : n; };
  std::vector<std::vector<int64_t>> hk_save(T);
  std::vector<std::vector<uint64_t>> hw_save(T);
  auto save_head = [&](int g) {
    const uint64_t a = start_of(g), h = std::min(r0[g], start_of(g + 1) - a);
    hk_save[g].assign(keys + a, keys + a + h);
    hw_save[g].assign(aggs + a * na, aggs + (a + h) * na);
  };
  auto run_group = [&](int g) {
    const uint64_t a = start_of(g), h = hk_save[g].size();
    uint64_t end = start_of(g + 1);
    for (uint64_t r = r0[g + 1]; r-- > r0[g];) {
      const uint64_t p = pos[r], j = fresh_j[r];
      if (end > p) {
        const uint64_t mem0 = std::max(p, a + h);  // rows [p, a + h) come from the saved head
        if (end > mem0) move_rows(mem0, mem0 + r + 1, end - mem0);
        for (uint64_t i = p; i < std::min(end, a + h); ++i) {
          keys[i + r + 1] = hk_save[g][i - a];
          memcpy(aggs + (i + r + 1) * na, &hw_save[g][(i - a) * na], (size_t)na * 8);
        }
      }
      keys[p + r] = hk[j];
      memcpy(aggs + (p + r) * na, &hw[j * na], (size_t)na * 8);
      end = p;
    }
  };
  if (T <= 1) {
    hk_save.resize(1);
    hw_save.resize(1);
    if (T == 1) run_group(0);  // (group 0's head is never written by another group: no copy)
  } else {
    std::vector<std::thread> th;
    for (int g = 1; g < T; ++g) th.emplace_back(save_head, g);
    for (auto &t : th) t.join();
    th.clear();
    for (int g = 0; g < T; ++g) th.emplace_back(run_group, g);
    for (auto &t : th) t.join();
  }
  return n + fresh;
}

}  // namespace fold
}  // namespace nut
