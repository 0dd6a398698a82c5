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

// One thread: publish this tile's aggregate (tile 0: its inclusive prefix) as soon as it is
// known, before anything waits — so that every tile holding a ticket publishes in bounded
// time, and a workgroup may take its next tile before resolving this one.
__device__ inline void lookback_publish(uint64_t *__restrict__ status, uint32_t tile, uint64_t total) {
  st_agent(&status[tile], (tile == 0 ? FLAG_INC : FLAG_AGG) | total);
}

// One wave, after lookback_publish: this tile's exclusive prefix; publishes its inclusive one.
// Each lane reads LB_PER consecutive predecessors, so one step of the walk covers
// 64 * LB_PER tiles.
constexpr int LB_PER = 1;  // 4 was measured slower (filter 0.2945 vs 0.2780 ms, scripts/tune/filter_tune.hip "LB4")
__device__ inline uint64_t lookback_resolve(uint64_t *__restrict__ status, uint32_t tile, uint64_t total,
                                            uint32_t *__restrict__ err, int lane) {
  if (tile == 0) return 0;
  uint64_t excl = 0;
  int64_t pred = (int64_t)tile - 1;
  uint32_t spins = 0;
  for (;;) {
    uint64_t s[LB_PER];  // s[k] = status[pred - LB_PER * lane - k]: k = 0 is the most recent
#pragma unroll
    for (int k = 0; k < LB_PER; ++k) {
      const int64_t idx = pred - LB_PER * lane - k;
      s[k] = idx >= 0 ? ld_agent(&status[idx]) : FLAG_INC;
    }
    for (;;) {
      bool wait = false;
#pragma unroll
      for (int k = 0; k < LB_PER; ++k) wait |= (s[k] >> 62) == 0;
      if (!__any(wait)) break;
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int k = 0; k < LB_PER; ++k)
        if ((s[k] >> 62) == 0) s[k] = ld_agent(&status[pred - LB_PER * lane - k]);
      if (++spins > SPIN_LIMIT) {  // never expected: predecessors always run ahead
        if (lane == 0) atomicOr(err, 1u);
#pragma unroll
        for (int k = 0; k < LB_PER; ++k) s[k] = FLAG_INC | (s[k] & VAL_MASK);
      }
    }
    // this lane's share up to (and including) its most recent inclusive prefix, if any
    uint64_t mine = 0;
    bool inc = false;
#pragma unroll
    for (int k = 0; k < LB_PER; ++k) {
      if (!inc) mine += s[k] & VAL_MASK;
      inc |= (s[k] >> 62) == 2;
    }
    const uint64_t incs = __ballot(inc);
    if (incs) {
      const int first = __builtin_ctzll(incs);
      excl += wave_sum_u64(lane <= first ? mine : 0);
      break;
    }
    excl += wave_sum_u64(mine);
    pred -= kWave * LB_PER;
  }
  if (lane == 0) st_agent(&status[tile], FLAG_INC | (excl + total));
  return excl;
}

// Wave 0 of the block: publish this tile's aggregate and return its exclusive prefix.
__device__ inline uint64_t lookback(uint64_t *__restrict__ status, uint32_t tile, uint64_t total,
                                    uint32_t *__restrict__ err, int lane) {
  if (lane == 0) lookback_publish(status, tile, total);
  return lookback_resolve(status, tile, total, err, lane);
}

}  // namespace nut
