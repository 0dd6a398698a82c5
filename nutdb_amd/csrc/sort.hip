// sort.hip — SELECT k FROM t ORDER BY k  (BASELINE config 5): LSD radix sort of int64.
//
// Onesweep-style:
//   * keys are mapped to u64 with the sign bit flipped (order-preserving); 8 passes of
//     8-bit digits, least significant first; a pass whose digit is constant over all
//     keys (one histogram bin = n) is skipped;
//   * ONE upfront read computes all eight 256-bin histograms (LDS per block, then
//     global atomics); a tiny kernel turns them into per-pass digit bases;
//   * per pass ONE kernel: a 4096-key tile (256 threads = 4 waves x 16 items) is ranked
//     stably in registers — peers of a key within its wave from 8 ballots over the
//     digit bits, running per-wave digit counters in LDS — then every digit's tile
//     offset comes from a decoupled look-back (thread t owns digit t; 8-B {flag|count}
//     granules, relaxed agent-scope stores/loads, no fence), and the tile is staged in
//     LDS in digit order so consecutive threads write consecutive addresses of a bucket.
// Algorithmic bytes: 8 B/key histogram read + 16 B/key per executed pass.
#include <string.h>

#include <algorithm>

#include "common.hpp"

namespace nut {

constexpr int RS_THREADS = 256;
constexpr int RS_WAVES = RS_THREADS / kWave;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;  // 4096 keys
constexpr int RS_BINS = 256;
constexpr uint64_t RS_FLIP = 0x8000000000000000ull;      // ascending: signed order -> unsigned order
constexpr uint64_t RS_FLIP_DESC = 0x7FFFFFFFFFFFFFFFull; // descending: the complement of the above
constexpr uint64_t RS_AGG = 1ull << 62;
constexpr uint64_t RS_INC = 2ull << 62;
constexpr uint64_t RS_VAL = (1ull << 62) - 1;
constexpr uint32_t RS_SPIN_LIMIT = 1u << 24;
constexpr int RS_LBW = 8;  // predecessor granules per look-back round trip

// ---------------------------------------------------------------- histograms
__global__ __launch_bounds__(RS_THREADS) void rs_hist_kernel(const int64_t *__restrict__ in, uint64_t n, uint64_t flip,
                                                             unsigned long long *__restrict__ hist) {
  __shared__ uint32_t h[8][RS_BINS];
  for (int i = threadIdx.x; i < 8 * RS_BINS; i += RS_THREADS) (&h[0][0])[i] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * RS_THREADS * 2;
  for (uint64_t i = ((uint64_t)blockIdx.x * RS_THREADS + threadIdx.x) * 2; i < n; i += stride) {
    uint64_t a, b;
    bool two = i + 1 < n;
    if (two && ((((uintptr_t)(in + i)) & 15) == 0)) {
      const u64x2 v = *reinterpret_cast<const u64x2 *>(in + i);
      a = v.x;
      b = v.y;
    } else {
      a = (uint64_t)in[i];
      b = two ? (uint64_t)in[i + 1] : 0;
    }
    a ^= flip;
    b ^= flip;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      atomicAdd(&h[p][(a >> (8 * p)) & 255], 1u);
      if (two) atomicAdd(&h[p][(b >> (8 * p)) & 255], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 8 * RS_BINS; i += RS_THREADS) {
    uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&hist[i], (unsigned long long)c);
  }
}

// exclusive scan of each pass's 256 bins -> digit bases; flags passes whose digit is
// constant (skippable).  One block per pass.
__global__ __launch_bounds__(RS_BINS) void rs_scan_kernel(const unsigned long long *__restrict__ hist, uint64_t n,
                                                          uint64_t *__restrict__ base, uint32_t *__restrict__ trivial) {
  __shared__ uint64_t s[RS_BINS];
  const int p = blockIdx.x, t = threadIdx.x;
  const uint64_t c = hist[p * RS_BINS + t];
  s[t] = c;
  __syncthreads();
  if (t == 0) {
    uint64_t run = 0;
    bool triv = false;
    for (int i = 0; i < RS_BINS; ++i) {
      const uint64_t x = s[i];
      if (x == n) triv = true;
      s[i] = run;
      run += x;
    }
    trivial[p] = triv ? 1u : 0u;
  }
  __syncthreads();
  base[p * RS_BINS + t] = s[t];
}

// ---------------------------------------------------------------- one pass
// lanes of this wave holding the same digit (valid lanes only)
__device__ __forceinline__ uint64_t digit_peers(uint32_t d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint64_t bb = __ballot((d >> b) & 1u);
    m &= ((d >> b) & 1u) ? bb : ~bb;
  }
  return m;
}

// FIRST: input is raw int64 (flip on load); LAST: write int64 (flip back)
template <bool FIRST, bool LAST>
__global__ __launch_bounds__(RS_THREADS) void rs_pass_kernel(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                             uint64_t n, int shift, uint64_t flip,
                                                             const uint64_t *__restrict__ dbase,
                                                             uint64_t *__restrict__ status,
                                                             uint32_t *__restrict__ err) {
  __shared__ uint64_t s_keys[RS_TILE];             // tile staged in digit order
  __shared__ uint32_t s_wcnt[RS_WAVES][RS_BINS];    // per-wave digit counters -> wave prefixes
  __shared__ uint32_t s_tex[RS_BINS];              // exclusive digit offsets inside the tile
  __shared__ uint64_t s_gbase[RS_BINS];            // global position of the tile's first key of digit d

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < RS_WAVES * RS_BINS; i += RS_THREADS) (&s_wcnt[0][0])[i] = 0;
  // tile = blockIdx.x: workgroups are dispatched in ID order, so a tile only waits on
  // tiles dispatched before it (no global ticket: one contended atomic per tile cost
  // more than the look-back itself, see filter.hip)
  const uint32_t tile = blockIdx.x;
  const uint64_t tbase = (uint64_t)tile * RS_TILE;
  // wave w owns keys [w*ITEMS*64, (w+1)*ITEMS*64) of the tile; item i, lane l -> +i*64+l
  const uint64_t wbase = tbase + (uint64_t)wave * RS_ITEMS * kWave;

  uint64_t key[RS_ITEMS];
  uint32_t rank[RS_ITEMS];
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    const uint64_t idx = wbase + (uint64_t)i * kWave + lane;
    uint64_t k = idx < n ? in[idx] : 0;
    if (FIRST) k ^= flip;
    key[i] = k;
  }
  // stable in-wave ranking, items in order
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    const uint64_t idx = wbase + (uint64_t)i * kWave + lane;
    const bool valid = idx < n;
    const uint32_t d = (uint32_t)(key[i] >> shift) & 255u;
    const uint64_t peers = digit_peers(d, valid);
    const uint32_t before = lane_rank(peers);
    const uint32_t cnt = (uint32_t)__popcll(peers);
    uint32_t prior = valid ? s_wcnt[wave][d] : 0u;  // all peers read before the leader writes
    rank[i] = prior + before;
    if (valid && before == 0) s_wcnt[wave][d] = prior + cnt;
  }
  __syncthreads();
  // per digit (thread t = digit): tile count, wave prefixes, tile-internal offsets
  const int d = tid;
  uint32_t tot = 0;
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w) {
    const uint32_t c = s_wcnt[w][d];
    s_wcnt[w][d] = tot;  // exclusive prefix over waves
    tot += c;
  }
  // exclusive scan of tile counts over digits (block scan of 256 values)
  {
    uint32_t v = tot;
    // inclusive wave scan
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      uint32_t y = __shfl_up(v, off, 64);
      if (lane >= off) v += y;
    }
    __shared__ uint32_t s_wsum[RS_WAVES];
    if (lane == 63) s_wsum[wave] = v;
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) add += (w < wave) ? s_wsum[w] : 0u;
    s_tex[d] = v - tot + add;
  }
  // decoupled look-back, thread d walks back through predecessors' digit-d granules
  {
    uint64_t *my = &status[(uint64_t)tile * RS_BINS + d];
    uint64_t excl = 0;
    if (tile == 0) {
      st_agent(my, RS_INC | tot);
    } else {
      st_agent(my, RS_AGG | tot);
      // walk back RS_LBW predecessors per round trip (loads issued together)
      int64_t j = (int64_t)tile - 1;
      uint32_t spins = 0;
      bool done = false;
      while (!done) {
        uint64_t sv[RS_LBW];
#pragma unroll
        for (int m = 0; m < RS_LBW; ++m)
          sv[m] = j - m >= 0 ? ld_agent(&status[(uint64_t)(j - m) * RS_BINS + d]) : RS_INC;
#pragma unroll
        for (int m = 0; m < RS_LBW; ++m) {
          if (done) break;
          uint64_t sm = sv[m];
          while ((sm >> 62) == 0) {
            __builtin_amdgcn_s_sleep(1);
            sm = ld_agent(&status[(uint64_t)(j - m) * RS_BINS + d]);
            if (++spins > RS_SPIN_LIMIT) {
              atomicOr(err, 1u);
              sm = RS_INC;
            }
          }
          excl += sm & RS_VAL;
          if ((sm >> 62) == 2) done = true;
        }
        j -= RS_LBW;
      }
      st_agent(my, RS_INC | (excl + tot));
    }
    s_gbase[d] = dbase[d] + excl;
  }
  __syncthreads();
  // stage in digit order
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    const uint64_t idx = wbase + (uint64_t)i * kWave + lane;
    if (idx < n) {
      const uint32_t dd = (uint32_t)(key[i] >> shift) & 255u;
      s_keys[s_tex[dd] + s_wcnt[wave][dd] + rank[i]] = key[i];
    }
  }
  __syncthreads();
  // write: consecutive threads -> consecutive positions inside each digit's run
  const uint32_t valid_n = (uint32_t)min<uint64_t>(RS_TILE, n - tbase);
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    const uint32_t j = (uint32_t)i * RS_THREADS + tid;
    if (j < valid_n) {
      const uint64_t k = s_keys[j];
      const uint32_t dd = (uint32_t)(k >> shift) & 255u;
      out[s_gbase[dd] + (j - s_tex[dd])] = LAST ? (k ^ flip) : k;
    }
  }
}

__global__ void rs_copy_kernel(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

}  // namespace nut

using namespace nut;

static nut_status sort_i64(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n, uint64_t flip) {
  if (!c || (n && (!in || !out))) return fail(NUT_ERR_INVALID_ARG, "nut_sort_i64: NULL argument");
  if (n && (uintptr_t)in == (uintptr_t)out) return fail(NUT_ERR_INVALID_ARG, "nut_sort_i64: in and out alias");
  if (n == 0) return NUT_OK;
  DeviceGuard g(c->device);
  const uint64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  if (ntiles > 0xFFFFFFF0ull) return fail(NUT_ERR_UNSUPPORTED, "nut_sort_i64: n too large");
  // scratch: [pad+err 16 B | status ntiles*256*8 | hist 8*256*8 | base 8*256*8 | trivial 8*4
  //           | ping-pong buffer n*8]
  const size_t st_bytes = 16 + ntiles * RS_BINS * 8;
  const size_t o_hist = (st_bytes + 255) & ~size_t(255);
  const size_t o_base = o_hist + 8 * RS_BINS * 8;
  const size_t o_triv = o_base + 8 * RS_BINS * 8;
  const size_t o_tmp = (o_triv + 64 + 255) & ~size_t(255);
  nut_status s = c->sort_tmp.reserve(o_tmp + n * 8);
  if (s) return s;
  char *b = (char *)c->sort_tmp.ptr;
  uint32_t *err = (uint32_t *)(b + o_triv + 32);  // survives the per-pass memset
  uint64_t *status = (uint64_t *)(b + 16);
  unsigned long long *hist = (unsigned long long *)(b + o_hist);
  uint64_t *base = (uint64_t *)(b + o_base);
  uint32_t *triv = (uint32_t *)(b + o_triv);
  uint64_t *tmp = (uint64_t *)(b + o_tmp);
  hipStream_t st = c->stream;

  c->timer.begin(st, NUT_KERNEL_SORT);
  NUT_HIP(hipMemsetAsync(hist, 0, 8 * RS_BINS * 8, st));
  NUT_HIP(hipMemsetAsync(err, 0, 4, st));
  uint64_t hblocks = std::min<uint64_t>((n + 2 * RS_THREADS - 1) / (2 * RS_THREADS), (uint64_t)c->num_cus * 4);
  hipLaunchKernelGGL(rs_hist_kernel, dim3((unsigned)hblocks), dim3(RS_THREADS), 0, st, in, n, flip, hist);
  hipLaunchKernelGGL(rs_scan_kernel, dim3(8), dim3(RS_BINS), 0, st, (const unsigned long long *)hist, n, base, triv);
  NUT_HIP(hipGetLastError());
  // which passes run is decided on the host (8 flags)
  uint32_t htriv[8];
  NUT_HIP(hipMemcpyAsync(htriv, triv, sizeof(htriv), hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  int passes[8], np = 0;
  for (int p = 0; p < 8; ++p)
    if (!htriv[p]) passes[np++] = p;
  if (np == 0) {  // all keys equal
    hipLaunchKernelGGL(rs_copy_kernel, dim3((unsigned)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256), 0, st,
                       (const uint64_t *)in, (uint64_t *)out, n);
    c->timer.end(st);
    NUT_HIP(hipGetLastError());
    return NUT_OK;
  }
  // ping-pong so that the last executed pass writes `out`
  const uint64_t *src = (const uint64_t *)in;
  for (int k = 0; k < np; ++k) {
    const bool first = k == 0, last = k == np - 1;
    uint64_t *dst = ((np - 1 - k) % 2 == 0) ? (uint64_t *)out : tmp;
    NUT_HIP(hipMemsetAsync(b, 0, st_bytes, st));
    const int p = passes[k];
    const uint64_t *db = base + p * RS_BINS;
    auto kern = first ? (last ? rs_pass_kernel<true, true> : rs_pass_kernel<true, false>)
                      : (last ? rs_pass_kernel<false, true> : rs_pass_kernel<false, false>);
    hipLaunchKernelGGL(kern, dim3((unsigned)ntiles), dim3(RS_THREADS), 0, st, src, dst, n, 8 * p, flip, db, status,
                       err);
    NUT_HIP(hipGetLastError());
    src = dst;
  }
  c->timer.end(st);
  NUT_HIP(hipMemcpyAsync(htriv, err, 4, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  if (htriv[0]) return fail(NUT_ERR_TIMEOUT, "nut_sort_i64: look-back spin limit hit");
  return NUT_OK;
}

extern "C" nut_status nut_sort_i64(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n) {
  return sort_i64(c, in, out, n, RS_FLIP);
}

extern "C" nut_status nut_sort_i64_desc(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n) {
  return sort_i64(c, in, out, n, RS_FLIP_DESC);
}
