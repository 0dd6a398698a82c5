// filter.hip — SELECT col FROM t WHERE col <op> k  (BASELINE config 2)
//
// One pass over the column, order-preserving stream compaction:
//   * 512-thread workgroups, one 16384-row tile each (16 stripes x 16 B per lane, a
//     wave instruction reads 1 KiB contiguous; non-temporal loads: the column is
//     streamed once).  Tile order comes from an atomic ticket taken at workgroup start,
//     so a tile only ever waits on tiles that are already running, whatever the dispatch
//     order (cdna_hip_programming.md §6 G16: no dependence on dispatch order).  The
//     ticket serialises on one address: 0.11 ms at 24414 tiles, hence the large tiles
//     (6104 tiles at N = 1e8; ~5 % of the kernel, scripts/tune/filter_tune.hip).
//   * in-wave rank: __ballot + v_mbcnt (no shuffles); cross-wave: 16x8 counts in LDS.
//   * the comparison is a template parameter (no per-row switch).
//   * global offset: single-pass decoupled look-back.  Each tile publishes ONE 8-byte
//     granule {flag:2 | count:62} with a relaxed agent-scope (sc1) store; predecessors
//     are read by one wave, 64 tiles per step, with relaxed agent-scope loads — the
//     data is its own flag, so no fence is needed (cdna_hip_programming.md §6 G16, R2).
//   * selected values are stored straight to their final position (L2 merges the
//     partial lines before write-back).
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
  uint64_t ntiles = (n + FT_TILE - 1) / FT_TILE;
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
  bool aligned = ((uintptr_t)col & 15) == 0;
  c->timer.begin(c->stream, NUT_KERNEL_FILTER);
  using K = void (*)(const int64_t *, uint64_t, int64_t, int64_t *, uint64_t *, uint32_t *, uint64_t *, uint32_t,
                     uint32_t *);
  static const K kern[2][6] = {
      {filter_i64_kernel<false, NUT_LT>, filter_i64_kernel<false, NUT_LE>, filter_i64_kernel<false, NUT_GT>,
       filter_i64_kernel<false, NUT_GE>, filter_i64_kernel<false, NUT_EQ>, filter_i64_kernel<false, NUT_NE>},
      {filter_i64_kernel<true, NUT_LT>, filter_i64_kernel<true, NUT_LE>, filter_i64_kernel<true, NUT_GT>,
       filter_i64_kernel<true, NUT_GE>, filter_i64_kernel<true, NUT_EQ>, filter_i64_kernel<true, NUT_NE>}};
  hipLaunchKernelGGL(kern[aligned ? 1 : 0][op], dim3((unsigned)ntiles), dim3(FT_THREADS), 0, c->stream, col, n, k,
                     out, out_n_dev, ticket, status, (uint32_t)ntiles, err);
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
