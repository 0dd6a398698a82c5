// lookback.hpp — single-pass decoupled look-back for order-preserving outputs (filter
// compaction, join pairs).  Each tile publishes ONE 8-byte granule {flag:2 | value:62}
// with a relaxed agent-scope (sc1) store; predecessors are read by one wave, 64 tiles per
// step, with relaxed agent-scope loads — the data is its own flag, so no fence is needed
// (cdna_hip_programming.md §6 G16, R2).  Tiles take their order from an atomic ticket at
// workgroup start, so a tile only waits on tiles already running.
#pragma once

#include "common.hpp"

namespace nut {

constexpr uint64_t FLAG_AGG = 1ull << 62;
constexpr uint64_t FLAG_INC = 2ull << 62;
constexpr uint64_t VAL_MASK = (1ull << 62) - 1;
constexpr uint32_t SPIN_LIMIT = 1u << 24;

// Wave 0 of the block: publish this tile's aggregate and return its exclusive prefix.
__device__ inline uint64_t lookback(uint64_t *__restrict__ status, uint32_t tile, uint64_t total,
                             uint32_t *__restrict__ err, int lane) {
  if (tile == 0) {
    if (lane == 0) st_agent(&status[0], FLAG_INC | total);
    return 0;
  }
  if (lane == 0) st_agent(&status[tile], FLAG_AGG | total);
  uint64_t excl = 0;
  int64_t pred = (int64_t)tile - 1;
  uint32_t spins = 0;
  for (;;) {
    int64_t idx = pred - lane;
    uint64_t s = idx >= 0 ? ld_agent(&status[idx]) : FLAG_INC;
    while (__any((s >> 62) == 0)) {
      __builtin_amdgcn_s_sleep(1);
      if ((s >> 62) == 0) s = ld_agent(&status[idx]);
      if (++spins > SPIN_LIMIT) {  // never expected: predecessors always run ahead
        if (lane == 0) atomicOr(err, 1u);
        s = FLAG_INC | (s & VAL_MASK);
      }
    }
    uint64_t inc = __ballot((s >> 62) == 2);
    if (inc) {
      int first = __builtin_ctzll(inc);
      excl += wave_sum_u64(lane <= first ? (s & VAL_MASK) : 0);
      break;
    }
    excl += wave_sum_u64(s & VAL_MASK);
    pred -= kWave;
  }
  if (lane == 0) st_agent(&status[tile], FLAG_INC | (excl + total));
  return excl;
}

}  // namespace nut
