// filter.hip — SELECT col FROM t WHERE col <op> k  (BASELINE config 2)
//
// One pass over the column, order-preserving stream compaction.  Product kernel
// (filter_i64_staged_kernel, 16-B aligned columns of >= 2 rows, 8-B aligned output):
//   * persistent: one 1024-thread workgroup per CU, tiles of 32768 rows (16 stripes x
//     16 B per lane, a wave instruction reads 1 KiB contiguous, non-temporal loads) taken
//     from an atomic ticket, so a tile only ever waits on tiles that are already running,
//     whatever the dispatch order (cdna_hip_programming.md §6 G16).
//   * in-wave rank: __ballot + v_mbcnt; stripe bases: lane j of each wave sums stripe j's
//     per-wave counts and one 16-lane scan gives every (stripe, wave) start.
//   * the selected rows move from registers into an LDS buffer in tile order; the
//     registers are then free and take the NEXT tile's loads BEFORE this tile's global
//     offset is resolved, so the look-back round trips overlap HBM reads instead of
//     stalling them (measured: 0.285 -> 0.220 ms at N = 1e8, s = 0.5).
//   * global offset: single-pass decoupled look-back (lookback.hpp), one 8-byte granule
//     {flag:2 | count:62} per tile.
//   * the buffer is written out with aligned 16-B non-temporal stores (full lines).
//     A tile with more selected rows than the buffer holds stages and writes its two
//     halves in turn (no overlap for that tile).
// filter_i64_kernel (unaligned or tiny columns): one 16384-row tile per workgroup, values
// stored straight from registers after the look-back.
// Algorithmic bytes: 8 B/row read + 8 B/selected row written.
#include "common.hpp"
#include "lookback.hpp"

namespace nut {

constexpr int FT_THREADS = 512;
constexpr int FT_WAVES = FT_THREADS / kWave;               // 8
constexpr int FT_STRIPES = 16;                             // <= 16: selection bits fit a u32
constexpr int FT_STRIPE_ROWS = FT_THREADS * 2;             // 1024
constexpr int FT_TILE = FT_STRIPE_ROWS * FT_STRIPES;       // 16384 rows
template <bool FULL, bool ALIGNED>
__device__ __forceinline__ void load_stripe(const int64_t *__restrict__ col, uint64_t idx, uint64_t n,
                                            int64_t &a, int64_t &b) {
  if (FULL && ALIGNED) {
    i64x2 v = __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(col + idx));
    a = v.x;
    b = v.y;
  } else {
    a = (FULL || idx < n) ? col[idx] : 0;
    b = (FULL || idx + 1 < n) ? col[idx + 1] : 0;
  }
}

template <int OP>
__device__ __forceinline__ bool cmp_op(int64_t v, int64_t k) {
  return OP == NUT_LT ? v < k : OP == NUT_LE ? v <= k : OP == NUT_GT ? v > k : OP == NUT_GE ? v >= k
       : OP == NUT_EQ ? v == k : v != k;
}

template <bool ALIGNED, int OP>
__global__ __launch_bounds__(FT_THREADS) void filter_i64_kernel(
    const int64_t *__restrict__ col, uint64_t n, int64_t k, int64_t *__restrict__ out,
    uint64_t *__restrict__ out_n, uint32_t *__restrict__ ticket, uint64_t *__restrict__ status,
    uint32_t ntiles, uint32_t *__restrict__ err) {
  __shared__ uint32_t s_cnt[FT_STRIPES][FT_WAVES];
  __shared__ uint64_t s_excl;
  __shared__ uint32_t s_tile;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(ticket, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t base = (uint64_t)tile * FT_TILE;
  const bool full = base + FT_TILE <= n;

  int64_t v0[FT_STRIPES], v1[FT_STRIPES];
  if (full) {
#pragma unroll
    for (int j = 0; j < FT_STRIPES; ++j)
      load_stripe<true, ALIGNED>(col, base + j * FT_STRIPE_ROWS + 2 * tid, n, v0[j], v1[j]);
  } else {
#pragma unroll
    for (int j = 0; j < FT_STRIPES; ++j)
      load_stripe<false, ALIGNED>(col, base + j * FT_STRIPE_ROWS + 2 * tid, n, v0[j], v1[j]);
  }

  // per stripe: in-wave rank of each of the lane's two rows
  uint32_t r0[FT_STRIPES];
  uint32_t sel = 0;  // bit 2j: row0 of stripe j selected, bit 2j+1: row1
#pragma unroll
  for (int j = 0; j < FT_STRIPES; ++j) {
    uint64_t idx = base + j * FT_STRIPE_ROWS + 2 * tid;
    bool p0 = cmp_op<OP>(v0[j], k) && (full || idx < n);
    bool p1 = cmp_op<OP>(v1[j], k) && (full || idx + 1 < n);
    uint64_t b0 = __ballot(p0), b1 = __ballot(p1);
    r0[j] = lane_rank(b0) + lane_rank(b1);
    sel |= (p0 ? 1u : 0u) << (2 * j);
    sel |= (p1 ? 1u : 0u) << (2 * j + 1);
    if (lane == 0) s_cnt[j][wave] = (uint32_t)(__popcll(b0) + __popcll(b1));
  }
  __syncthreads();

  if (wave == 0) {
    uint32_t c = 0;
#pragma unroll
    for (int i = lane; i < FT_STRIPES * FT_WAVES; i += kWave) c += (&s_cnt[0][0])[i];
    uint64_t total = wave_sum_u64(c);
    uint64_t excl = lookback(status, tile, total, err, lane);
    if (lane == 0) {
      s_excl = excl;
      if (tile == ntiles - 1) *out_n = excl + total;
    }
  }
  __syncthreads();
  uint64_t off = s_excl;
#pragma unroll
  for (int j = 0; j < FT_STRIPES; ++j) {
    uint64_t before = 0;
#pragma unroll
    for (int w = 0; w < FT_WAVES; ++w) before += (w < wave) ? s_cnt[j][w] : 0u;
    uint64_t pos = off + before + r0[j];
    bool p0 = (sel >> (2 * j)) & 1u, p1 = (sel >> (2 * j + 1)) & 1u;
    if (p0) out[pos] = v0[j];
    if (p1) out[pos + (p0 ? 1 : 0)] = v1[j];
#pragma unroll
    for (int w = 0; w < FT_WAVES; ++w) off += s_cnt[j][w];
  }
}


// ---- persistent, LDS-staged product kernel ----
constexpr int FS_THREADS = 1024;
constexpr int FS_WAVES = FS_THREADS / kWave;                // 16
constexpr int FS_STRIPES = 16;                              // stripe bases live in lanes 0..15
constexpr int FS_STRIPE_ROWS = FS_THREADS * 2;              // 2048
constexpr int FS_TILE = FS_STRIPE_ROWS * FS_STRIPES;        // 32768 rows
constexpr int FS_HALF = FS_TILE / 2;
constexpr int FS_CAP = 20224;                               // staged rows (158 KiB of LDS)
static_assert(FS_CAP >= FS_HALF, "a half tile must always fit the buffer");

// out[at .. at + cnt) = buf[0 .. cnt): aligned 16-B non-temporal stores, scalar head / tail
__device__ __forceinline__ void flush_staged(int64_t *__restrict__ out, uint64_t at, uint32_t cnt,
                                             const int64_t *buf, int tid) {
  const uint32_t head = (uint32_t)((((uintptr_t)(out + at)) >> 3) & 1);
  if (head && tid == 0 && cnt) out[at] = buf[0];
  for (uint32_t i = head + 2 * tid; i + 1 < cnt; i += 2 * FS_THREADS) {
    i64x2 w = {buf[i], buf[i + 1]};
    __builtin_nontemporal_store(w, reinterpret_cast<i64x2 *>(out + at + i));
  }
  if (cnt > head && ((cnt - head) & 1) && tid == FS_THREADS - 1) out[at + cnt - 1] = buf[cnt - 1];
}

template <int OP>
__global__ __launch_bounds__(FS_THREADS, 1) void filter_i64_staged_kernel(
    const int64_t *__restrict__ col, uint64_t n, int64_t k, int64_t *__restrict__ out,
    uint64_t *__restrict__ out_n, uint32_t *__restrict__ ticket, uint64_t *__restrict__ status,
    uint32_t ntiles, uint32_t *__restrict__ err) {
  __shared__ int64_t s_buf[FS_CAP];
  __shared__ uint32_t s_cnt[FS_STRIPES][FS_WAVES];
  __shared__ uint32_t s_next;
  __shared__ uint64_t s_excl;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  i64x2 v[FS_STRIPES];
  // one code path: 16-B loads at row indices clamped to n - 2 (n >= 2); rows >= n are
  // masked in the rank.  Only the pair (n - 1, n) of an odd n is clamped while holding a
  // valid row: it loads (n - 2, n - 1) and takes its row from the upper half — when the
  // tile is ranked, not at the load: a select on a loaded value waits for it,
  // and the next tile's loads, issued before this tile's write-out, would all be waited
  // for before that write-out could start (vmcnt is in order)
  auto load = [&](uint32_t t) {
    const uint64_t base = (uint64_t)t * FS_TILE;
#pragma unroll
    for (int j = 0; j < FS_STRIPES; ++j) {
      const uint64_t idx = min(base + j * FS_STRIPE_ROWS + 2 * tid, n - 2);
      v[j] = __builtin_nontemporal_load(reinterpret_cast<const i64x2 *>(col + idx));
    }
  };

  if (tid == 0) s_next = atomicAdd(ticket, 1u);
  __syncthreads();
  uint32_t tile = s_next;
  if (tile >= ntiles) return;
  load(tile);
  for (;;) {
    // an opaque copy of tid per tile: hoisted out of the loop, the per-stripe row offsets
    // pinned registers the stripes need (spills)
    int tid_ = tid;
    asm volatile("" : "+v"(tid_));
    const int tid = tid_;
    const uint64_t base = (uint64_t)tile * FS_TILE;
    const bool full = base + FS_TILE <= n;
    if (!full) {  // (the last tile only) the pair holding row n - 1 alone takes its upper half
      const uint64_t r = n - 1 - base;
      const bool mine = (r & 1) == 0 && (uint32_t)((r % FS_STRIPE_ROWS) / 2) == (uint32_t)tid;
      const uint32_t js = (uint32_t)(r / FS_STRIPE_ROWS);
#pragma unroll
      for (int j = 0; j < FS_STRIPES; ++j) v[j].x = mine && js == (uint32_t)j ? v[j].y : v[j].x;
    }
    uint32_t rk[FS_STRIPES / 4] = {};  // in-wave ranks (<= 126), 4 per word
    uint32_t sel = 0;                  // bit 2j: row0 of stripe j selected, bit 2j+1: row1
#pragma unroll
    for (int j = 0; j < FS_STRIPES; ++j) {
      const uint64_t idx = base + j * FS_STRIPE_ROWS + 2 * tid;
      const bool p0 = cmp_op<OP>(v[j].x, k) && (full || idx < n);
      const bool p1 = cmp_op<OP>(v[j].y, k) && (full || idx + 1 < n);
      const uint64_t b0 = __ballot(p0), b1 = __ballot(p1);
      rk[j / 4] |= (lane_rank(b0) + lane_rank(b1)) << (8 * (j % 4));
      sel |= (p0 ? 1u : 0u) << (2 * j);
      sel |= (p1 ? 1u : 0u) << (2 * j + 1);
      if (lane == 0) s_cnt[j][wave] = (uint32_t)(__popcll(b0) + __popcll(b1));
    }
    if (tid == kWave) s_next = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tn = s_next;
    // lane j < 16: stripe j's total T and the part of it in waves before this one (P)
    uint32_t T = 0, P = 0;
    if (lane < FS_STRIPES) {
#pragma unroll
      for (int w = 0; w < FS_WAVES; ++w) {
        const uint32_t c = s_cnt[lane][w];
        T += c;
        P += w < wave ? c : 0u;
      }
    }
    uint32_t incl = T;
#pragma unroll
    for (int d = 1; d < FS_STRIPES; d <<= 1) {
      const uint32_t o = __shfl_up(incl, d, kWave);
      incl += lane >= d ? o : 0u;
    }
    const uint32_t pre = incl - T + P;  // tile-local start of this wave's rows of stripe `lane`
    const uint32_t total = __builtin_amdgcn_readlane(incl, FS_STRIPES - 1);
    const uint32_t half = __builtin_amdgcn_readlane(incl, FS_STRIPES / 2 - 1);  // rows of stripes 0..7
    const bool fits = total <= FS_CAP;  // uniform
    auto stage = [&](int j0, int j1, uint32_t shift) {
#pragma unroll
      for (int j = 0; j < FS_STRIPES; ++j) {
        if (j < j0 || j >= j1) continue;
        const uint32_t pos = __builtin_amdgcn_readlane(pre, j) - shift + ((rk[j / 4] >> (8 * (j % 4))) & 0xFFu);
        const bool p0 = (sel >> (2 * j)) & 1u, p1 = (sel >> (2 * j + 1)) & 1u;
        if (p0) s_buf[pos] = v[j].x;
        if (p1) s_buf[pos + (p0 ? 1 : 0)] = v[j].y;
      }
    };
    auto resolve = [&]() {
      if (wave == 0) {
        const uint64_t excl = lookback(status, tile, total, err, lane);
        if (lane == 0) {
          s_excl = excl;
          if (tile == ntiles - 1) *out_n = excl + total;
        }
      }
    };
    if (fits) {
      stage(0, FS_STRIPES, 0);
    } else {  // dense tile: stage and write the first half before the registers are freed
      stage(0, FS_STRIPES / 2, 0);
      resolve();
      __syncthreads();
      flush_staged(out, s_excl, half, s_buf, tid);
      __syncthreads();
      stage(FS_STRIPES / 2, FS_STRIPES, half);
    }
    __builtin_amdgcn_sched_barrier(0);  // the registers are free from here on
    if (fits) resolve();                // wave 0 walks before it has data loads in flight
    if (tn < ntiles) load(tn);
    __syncthreads();
    if (fits)
      flush_staged(out, s_excl, total, s_buf, tid);
    else
      flush_staged(out, s_excl + half, total - half, s_buf, tid);
    if (tn >= ntiles) break;
    tile = tn;
  }
}
}  // namespace nut

using namespace nut;

extern "C" nut_status nut_filter_i64_async(nut_ctx *c, const int64_t *col, uint64_t n, int op,
                                           int64_t k, int64_t *out, uint64_t *out_n_dev) {
  if (!c || !out_n_dev || (n && (!col || !out)))
    return fail(NUT_ERR_INVALID_ARG, "nut_filter_i64: NULL argument");
  if (op < NUT_LT || op > NUT_NE) return fail(NUT_ERR_INVALID_ARG, "nut_filter_i64: bad cmp op");
  DeviceGuard g(c->device);
  if (n == 0) {
    NUT_HIP(hipMemsetAsync(out_n_dev, 0, sizeof(uint64_t), c->stream));
    return NUT_OK;
  }
  const bool aligned = ((uintptr_t)col & 15) == 0 && ((uintptr_t)out & 7) == 0;
  const bool staged = aligned && n >= 2;
  const uint64_t tile_rows = staged ? FS_TILE : FT_TILE;
  uint64_t ntiles = (n + tile_rows - 1) / tile_rows;
  if (ntiles > 0xFFFFFFF0ull) return fail(NUT_ERR_UNSUPPORTED, "nut_filter_i64: n too large");
  // [ticket u32, err u32, pad 8][status u64 x ntiles] — zeroed each call as one block
  size_t state = 16 + ntiles * 8;
  state = (state + 15) & ~size_t(15);
  nut_status st = c->filter_state.reserve(state);
  if (st) return st;
  char *base = (char *)c->filter_state.ptr;
  uint32_t *ticket = (uint32_t *)base;
  uint32_t *err = ticket + 1;
  uint64_t *status = (uint64_t *)(base + 16);
  NUT_HIP(hipMemsetAsync(base, 0, state, c->stream));
  c->timer.begin(c->stream, NUT_KERNEL_FILTER);
  using K = void (*)(const int64_t *, uint64_t, int64_t, int64_t *, uint64_t *, uint32_t *, uint64_t *, uint32_t,
                     uint32_t *);
  static const K kern[2][6] = {
      {filter_i64_kernel<false, NUT_LT>, filter_i64_kernel<false, NUT_LE>, filter_i64_kernel<false, NUT_GT>,
       filter_i64_kernel<false, NUT_GE>, filter_i64_kernel<false, NUT_EQ>, filter_i64_kernel<false, NUT_NE>},
      {filter_i64_kernel<true, NUT_LT>, filter_i64_kernel<true, NUT_LE>, filter_i64_kernel<true, NUT_GT>,
       filter_i64_kernel<true, NUT_GE>, filter_i64_kernel<true, NUT_EQ>, filter_i64_kernel<true, NUT_NE>}};
  static const K staged_kern[6] = {filter_i64_staged_kernel<NUT_LT>, filter_i64_staged_kernel<NUT_LE>,
                                   filter_i64_staged_kernel<NUT_GT>, filter_i64_staged_kernel<NUT_GE>,
                                   filter_i64_staged_kernel<NUT_EQ>, filter_i64_staged_kernel<NUT_NE>};
  if (staged) {
    // persistent: one workgroup per CU (158 KiB of LDS each), tiles by ticket
    const unsigned grid = (unsigned)std::min<uint64_t>(ntiles, (uint64_t)c->num_cus);
    hipLaunchKernelGGL(staged_kern[op], dim3(grid), dim3(FS_THREADS), 0, c->stream, col, n, k, out, out_n_dev,
                       ticket, status, (uint32_t)ntiles, err);
  } else {
    hipLaunchKernelGGL(kern[((uintptr_t)col & 15) == 0 ? 1 : 0][op], dim3((unsigned)ntiles), dim3(FT_THREADS), 0,
                       c->stream, col, n, k, out, out_n_dev, ticket, status, (uint32_t)ntiles, err);
  }
  c->timer.end(c->stream);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

extern "C" nut_status nut_filter_i64(nut_ctx *c, const int64_t *col, uint64_t n, int op, int64_t k,
                                     int64_t *out, uint64_t *out_n_host) {
  if (!c || !out_n_host) return fail(NUT_ERR_INVALID_ARG, "nut_filter_i64: NULL argument");
  DeviceGuard g(c->device);
  nut_status st = c->misc.reserve(64);
  if (st) return st;
  uint64_t *dev_n = (uint64_t *)c->misc.ptr;
  st = nut_filter_i64_async(c, col, n, op, k, out, dev_n);
  if (st) return st;
  // err flag is the word after the ticket in filter_state (only if n > 0)
  if (n) NUT_HIP(hipMemcpyAsync(c->host_pinned + 1, (char *)c->filter_state.ptr + 4, 4,
                                hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipMemcpyAsync(c->host_pinned, dev_n, 8, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  if (n && (uint32_t)c->host_pinned[1] != 0)
    return fail(NUT_ERR_TIMEOUT, "nut_filter_i64: look-back spin limit hit");
  *out_n_host = c->host_pinned[0];
  return NUT_OK;
}
