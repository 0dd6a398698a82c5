// select_kernel.hpp — expression-mode scan + compaction:
//   SELECT ... FROM t WHERE <any expression program>
// The WHERE program is the same generated kProg shape the expression-mode group-by uses
// (jit.cpp: where(p, v, r, err)), compiled into this kernel with hipRTC.  The kernel writes
// the row ids of the selected rows in row order (order-preserving stream compaction): a
// 512-thread workgroup takes tiles of 16384 rows by atomic ticket, evaluates the program on
// 32 striped rows per lane (the generated code reads only the columns the program names)
// and ranks the selected rows with ballots.  A tile's state after evaluation is one
// selection word per lane, so the workgroup is persistent and one tile ahead: it publishes
// tile t's count, evaluates tile t+1 (its HBM reads), and only then resolves t's global
// offset by decoupled look-back (lookback.hpp) and writes t's row ids — the look-back
// round trips overlap the next tile's reads instead of idling the workgroup.  Callers
// gather any column through the row ids (nut_gather_u64: ascending ids, near-sequential).
#pragma once

#include "agg_ops.hpp"
#include "lookback.hpp"

namespace nut {

constexpr int SEL_THREADS = 512;
constexpr int SEL_WAVES = SEL_THREADS / kWave;
constexpr int SEL_ITEMS = 32;  // <= 32: selection bits fit a u32
constexpr uint32_t SEL_TILE = SEL_THREADS * SEL_ITEMS;

struct SelArgs {
  AggArgs a;                 // n, val_col[] (program columns), kc[] (constants)
  int64_t *out;              // selected row ids
  uint64_t *status;          // look-back granules, one per tile
  uint32_t *ticket;          // [0] tile ticket, [1] error bits (1: spin limit, 2: division by zero)
  unsigned long long *out_n; // total selected
  uint32_t ntiles;
};

template <class S>
__global__ __launch_bounds__(SEL_THREADS) void select_kernel(SelArgs sa) {
  __shared__ uint32_t s_cnt[2][SEL_ITEMS][SEL_WAVES];
  __shared__ uint32_t s_tile[2];
  __shared__ uint64_t s_excl;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const uint64_t n = sa.a.n;
  // evaluate tile t into a selection word; per-(item, wave) counts into s_cnt[b]
  auto eval = [&](uint32_t t, int b) -> uint32_t {
    const uint64_t base = (uint64_t)t * SEL_TILE + tid;
    uint32_t sel = 0;
    bool err = false;
#pragma unroll
    for (int i = 0; i < SEL_ITEMS; ++i) {
      const uint64_t r = base + (uint64_t)i * SEL_THREADS;
      const bool ok = r < n;
      uint64_t vv[S::MV > 0 ? S::MV : 1][1];
#pragma unroll
      for (int c = 0; c < S::MV; ++c) vv[c][0] = ok ? __builtin_nontemporal_load(sa.a.val_col[c] + r) : 0;
      bool e = false;
      const bool w = S::where(sa.a, vv, 0, e) && ok;
      err = err || (e && ok);
      sel |= (w ? 1u : 0u) << i;
      const uint64_t bb = __ballot(w);
      if (lane == 0) s_cnt[b][i][wave] = (uint32_t)__popcll(bb);
    }
    if (__any(err) && lane == 0) atomicOr(sa.ticket + 1, 2u);
    return sel;
  };
  if (tid == 0) s_tile[0] = atomicAdd(sa.ticket, 1u);
  __syncthreads();
  uint32_t tile = s_tile[0];
  if (tile >= sa.ntiles) return;
  int b = 0;
  uint32_t sel = eval(tile, b);
  for (;;) {
    __syncthreads();  // s_cnt[b] complete
    uint64_t total = 0;
    if (wave == 0) {
      uint32_t c = 0;
#pragma unroll
      for (int k = lane; k < SEL_ITEMS * SEL_WAVES; k += kWave) c += (&s_cnt[b][0][0])[k];
      total = wave_sum_u64(c);
      if (lane == 0) lookback_publish(sa.status, tile, total);
    }
    if (tid == kWave) s_tile[b ^ 1] = atomicAdd(sa.ticket, 1u);
    __syncthreads();
    const uint32_t next = s_tile[b ^ 1];
    const uint32_t sel_next = next < sa.ntiles ? eval(next, b ^ 1) : 0u;
    if (wave == 0) {
      const uint64_t excl = lookback_resolve(sa.status, tile, total, sa.ticket + 1, lane);
      if (lane == 0) {
        s_excl = excl;
        if (tile == sa.ntiles - 1) *sa.out_n = excl + total;
      }
    }
    __syncthreads();
    const uint64_t base = (uint64_t)tile * SEL_TILE + tid;
    uint64_t off = s_excl;
#pragma unroll
    for (int i = 0; i < SEL_ITEMS; ++i) {
      uint32_t before = 0, all = 0;
#pragma unroll
      for (int w = 0; w < SEL_WAVES; ++w) {
        before += w < wave ? s_cnt[b][i][w] : 0u;
        all += s_cnt[b][i][w];
      }
      const bool w = (sel >> i) & 1u;
      const uint64_t bb = __ballot(w);
      if (w) sa.out[off + before + lane_rank(bb)] = (int64_t)(base + (uint64_t)i * SEL_THREADS);
      off += all;
    }
    if (next >= sa.ntiles) break;
    tile = next;
    sel = sel_next;
    b ^= 1;
  }
}

// Computed projections (nut_eval_rows; SELECT a * b, CASE ..., toYYYYMMDD(d) FROM t ...):
// out[a][i] = the value program a of the same generated shape at row rows[i] (rows NULL:
// row i), valid[a][i] = its mask program (a CASE branch that yields NULL; 1 without one,
// and the value word 0 where it is 0).  One row per lane, grid-stride: the selected row ids
// ascend, so the column reads are near-sequential; each output is one coalesced store.
constexpr int EV_THREADS = 256;

struct EvalArgs {
  AggArgs a;                    // val_col[] (program columns), kc[] (constants)
  const int64_t *rows;          // row ids (NULL: row i)
  uint64_t m;                   // rows to evaluate
  uint64_t *out[NUT_MAX_AGGS];  // one 8-byte word per row and program
  uint8_t *valid[NUT_MAX_AGGS]; // NULL: not written
  uint32_t *err;                // bit 2: division by zero
  int32_t nout, pad_;
};

template <class S>
__global__ __launch_bounds__(EV_THREADS) void eval_kernel(EvalArgs ea) {
  bool err = false;
  const uint64_t stride = (uint64_t)gridDim.x * EV_THREADS;
  for (uint64_t i = (uint64_t)blockIdx.x * EV_THREADS + threadIdx.x; i < ea.m; i += stride) {
    const uint64_t r = ea.rows ? (uint64_t)ea.rows[i] : i;
    uint64_t vv[S::MV > 0 ? S::MV : 1][1];
#pragma unroll
    for (int c = 0; c < S::MV; ++c) vv[c][0] = ea.a.val_col[c][r];
#pragma unroll
    for (int a = 0; a < S::MA; ++a) {
      if (a >= ea.nout) break;
      bool e = false;
      const bool ok = S::valid(ea.a, a, vv, 0, e);
      const uint64_t w = ok ? S::value(ea.a, a, vv, 0, e) : 0ull;
      err = err || e;
      ea.out[a][i] = w;
      if (ea.valid[a]) ea.valid[a][i] = ok ? 1 : 0;
    }
  }
  if (__any(err) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(ea.err, 2u);
}

}  // namespace nut
