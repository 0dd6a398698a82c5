// sort.hip — SELECT k FROM t ORDER BY k  (BASELINE config 5): LSD radix sort of int64,
// and the stable bucket partition that is the local step of the multi-GPU sample sort.
//
// Onesweep-style:
//   * keys are mapped to u64 with the sign bit flipped (order-preserving; DESC uses the
//     complement); 8 passes of 8-bit digits, least significant first; a pass whose digit
//     is constant over all keys (one histogram bin = n) is skipped;
//   * ONE upfront read computes all eight 256-bin histograms (LDS per block, then
//     global atomics); a tiny kernel turns them into per-pass digit bases;
//   * per pass ONE kernel: an 8192-key tile (512 threads = 8 waves x 16 items) is ranked
//     stably in registers — peers of a key within its wave from 8 ballots over the
//     digit bits, running per-wave digit counters in LDS — then every digit's tile
//     offset comes from a decoupled look-back (thread t < 256 owns digit t; 8-B
//     {epoch|flag|count} granules, relaxed agent-scope stores/loads, no fence), and the
//     tile is staged in LDS in digit order so consecutive threads write consecutive
//     addresses of a bucket;
//   * tile order comes from a per-pass atomic ticket (progress never depends on dispatch
//     order, cdna_hip_programming.md §6 G16) and the status granules carry the pass
//     epoch, so no per-pass memset of the status array (312 MB per pass at 1.25e9 keys).
// Measured (scripts/tune/sort_tune.hip, one pass, 2.5e8 keys): 256x16 tiles 1.72 ms,
// 512x16 tiles 1.40 ms; without the look-back 0.91 ms.
// Algorithmic bytes: 8 B/key histogram read + 16 B/key per executed pass.
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "common.hpp"
#include "sort.hpp"

namespace nut {

constexpr int RS_THREADS = 512;
constexpr int RS_WAVES = RS_THREADS / kWave;     // 8
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;   // 8192 keys
constexpr int RS_BINS = 256;
constexpr int RS_HIST_THREADS = 256;
constexpr uint64_t RS_FLIP = 0x8000000000000000ull;      // ascending: signed order -> unsigned order
constexpr uint64_t RS_FLIP_DESC = 0x7FFFFFFFFFFFFFFFull; // descending: the complement of the above
// status granule: [epoch:8 | flag:2 | count:54]
constexpr int RS_EPOCH_SHIFT = 56;
constexpr uint64_t RS_AGG = 1ull << 54;
constexpr uint64_t RS_INC = 2ull << 54;
constexpr uint64_t RS_VAL = (1ull << 54) - 1;
constexpr uint32_t RS_SPIN_LIMIT = 1u << 24;
constexpr int RS_MAX_BUCKETS = 64;  // nut_partition_i64: up to 63 splitters

static_assert(RS_THREADS >= RS_BINS, "one thread per digit in the scan / look-back");

// ---------------------------------------------------------------- digits
struct RadixDigit {  // bits [shift, shift+8) of the (flipped) key
  int shift;
  static constexpr int BITS = 8;
  __device__ __forceinline__ uint32_t operator()(uint64_t k, const int64_t *) const {
    return (uint32_t)(k >> shift) & 255u;
  }
};

struct BucketDigit {  // #splitters <= key (signed), splitters ascending in LDS
  int nsplit;
  static constexpr int BITS = 6;
  __device__ __forceinline__ uint32_t operator()(uint64_t k, const int64_t *spl) const {
    // branch-free lower bound over <= 63 splitters
    uint32_t lo = 0;
#pragma unroll
    for (int step = RS_MAX_BUCKETS / 2; step >= 1; step >>= 1)
      if (lo + step <= (uint32_t)nsplit && spl[lo + step - 1] <= (int64_t)k) lo += step;
    return lo;
  }
};

// ---------------------------------------------------------------- histograms
__global__ __launch_bounds__(RS_HIST_THREADS) void rs_hist_kernel(const int64_t *__restrict__ in, uint64_t n,
                                                                  uint64_t flip, unsigned long long *__restrict__ hist) {
  __shared__ uint32_t h[8][RS_BINS];
  for (int i = threadIdx.x; i < 8 * RS_BINS; i += RS_HIST_THREADS) (&h[0][0])[i] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * RS_HIST_THREADS * 2;
  for (uint64_t i = ((uint64_t)blockIdx.x * RS_HIST_THREADS + threadIdx.x) * 2; i < n; i += stride) {
    uint64_t a, b;
    bool two = i + 1 < n;
    if (two && ((((uintptr_t)(in + i)) & 15) == 0)) {
      const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(in + i));
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
  for (int i = threadIdx.x; i < 8 * RS_BINS; i += RS_HIST_THREADS) {
    uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&hist[i], (unsigned long long)c);
  }
}

// bucket histogram for nut_partition_i64
__global__ __launch_bounds__(RS_HIST_THREADS) void pt_hist_kernel(const int64_t *__restrict__ in, uint64_t n,
                                                                  BucketDigit dig, const int64_t *__restrict__ splitters,
                                                                  unsigned long long *__restrict__ hist) {
  __shared__ uint32_t h[RS_MAX_BUCKETS];
  __shared__ int64_t spl[RS_MAX_BUCKETS];
  for (int i = threadIdx.x; i < RS_MAX_BUCKETS; i += RS_HIST_THREADS) {
    h[i] = 0;
    spl[i] = i < dig.nsplit ? splitters[i] : INT64_MAX;
  }
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * RS_HIST_THREADS + threadIdx.x; i < n; i += (uint64_t)gridDim.x * RS_HIST_THREADS)
    atomicAdd(&h[dig((uint64_t)in[i], spl)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i <= dig.nsplit; i += RS_HIST_THREADS)
    if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
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
template <int BITS>
__device__ __forceinline__ uint64_t digit_peers(uint32_t d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < BITS; ++b) {
    const uint64_t bb = __ballot((d >> b) & 1u);
    m &= ((d >> b) & 1u) ? bb : ~bb;
  }
  return m;
}

// FIRST: input is raw int64 (flip on load); LAST: write int64 (flip back).
// nbins: digits in use (256 for radix passes, #buckets for a partition).
// PAIRS: every key carries a 64-bit payload (vin -> vout, moved with it; vin == NULL on
// the first pass = the row ids 0..n-1) — the stable key + row id sort of ORDER BY with
// projected columns (nut_sort_pairs).
template <bool FIRST, bool LAST, class Digit, bool PAIRS = false>
__global__ __launch_bounds__(RS_THREADS) void rs_pass_kernel(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                             uint64_t n, Digit dig, const int64_t *__restrict__ splitters,
                                                             int nbins, uint64_t flip, const uint64_t *__restrict__ dbase,
                                                             uint64_t *__restrict__ status, uint32_t epoch,
                                                             uint32_t *__restrict__ ticket,
                                                             uint32_t *__restrict__ err,
                                                             const uint64_t *__restrict__ vin = nullptr,
                                                             uint64_t *__restrict__ vout = nullptr) {
  __shared__ uint64_t s_keys[RS_TILE];             // tile staged in digit order
  __shared__ uint64_t s_vals[PAIRS ? RS_TILE : 1];  // and its payload
  __shared__ uint32_t s_wcnt[RS_WAVES][RS_BINS];    // per-wave digit counters -> wave prefixes
  __shared__ uint32_t s_tex[RS_BINS];              // exclusive digit offsets inside the tile
  __shared__ uint64_t s_gbase[RS_BINS];            // global position of the tile's first key of digit d
  __shared__ uint32_t s_wsum[RS_BINS / kWave];
  __shared__ int64_t s_spl[RS_MAX_BUCKETS];
  __shared__ uint32_t s_tile;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < RS_WAVES * RS_BINS; i += RS_THREADS) (&s_wcnt[0][0])[i] = 0;
  if (splitters && tid < RS_MAX_BUCKETS) s_spl[tid] = tid < nbins - 1 ? splitters[tid] : INT64_MAX;
  // ticket: a tile only waits on tiles that already hold a ticket (running or done)
  if (tid == 0) s_tile = atomicAdd(ticket, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t tbase = (uint64_t)tile * RS_TILE;
  // wave w owns keys [w*ITEMS*64, (w+1)*ITEMS*64) of the tile; item i, lane l -> +i*64+l
  const uint64_t wbase = tbase + (uint64_t)wave * RS_ITEMS * kWave;

  uint64_t key[RS_ITEMS];
  uint64_t val[PAIRS ? RS_ITEMS : 1];
  uint32_t rank[RS_ITEMS];
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    const uint64_t idx = wbase + (uint64_t)i * kWave + lane;
    const uint64_t ci = idx < n ? idx : n - 1;  // clamped, unconditional: the loads overlap
    uint64_t k = in[ci];
    if (FIRST) k ^= flip;
    key[i] = k;
    if constexpr (PAIRS) val[i] = (FIRST && !vin) ? idx : vin[ci];
  }
  // stable in-wave ranking, items in order
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    const uint64_t idx = wbase + (uint64_t)i * kWave + lane;
    const bool valid = idx < n;
    const uint32_t d = dig(key[i], s_spl);
    const uint64_t peers = digit_peers<Digit::BITS>(d, valid);
    const uint32_t before = lane_rank(peers);
    const uint32_t cnt = (uint32_t)__popcll(peers);
    uint32_t prior = valid ? s_wcnt[wave][d] : 0u;  // all peers read before the leader writes
    rank[i] = prior + before;
    if (valid && before == 0) s_wcnt[wave][d] = prior + cnt;
  }
  __syncthreads();
  // per digit (thread t < 256 = digit): tile count and wave prefixes
  uint32_t tot = 0, incl = 0;
  if (tid < RS_BINS) {
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) {
      const uint32_t c = s_wcnt[w][tid];
      s_wcnt[w][tid] = tot;  // exclusive prefix over waves
      tot += c;
    }
    // inclusive scan of tile counts over digits: waves 0..3, then across them
    incl = tot;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      uint32_t y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) s_wsum[wave] = incl;
  }
  __syncthreads();
  if (tid < RS_BINS) {
    const int d = tid;
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < RS_BINS / kWave; ++w) add += (w < wave) ? s_wsum[w] : 0u;
    s_tex[d] = incl - tot + add;
    // decoupled look-back, thread d walks back through predecessors' digit-d granules
    uint64_t excl = 0;
    if (d < nbins) {
      const uint64_t ep = (uint64_t)epoch << RS_EPOCH_SHIFT;
      uint64_t *my = &status[(uint64_t)tile * RS_BINS + d];
      if (tile == 0) {
        st_agent(my, ep | RS_INC | tot);
      } else {
        st_agent(my, ep | RS_AGG | tot);
        int64_t j = (int64_t)tile - 1;
        uint32_t spins = 0;
        for (;;) {
          uint64_t s = ld_agent(&status[(uint64_t)j * RS_BINS + d]);
          while ((s >> RS_EPOCH_SHIFT) != epoch) {  // not yet published in this pass
            __builtin_amdgcn_s_sleep(1);
            s = ld_agent(&status[(uint64_t)j * RS_BINS + d]);
            if (++spins > RS_SPIN_LIMIT) {
              atomicOr(err, 1u);
              s = ep | RS_INC;
            }
          }
          excl += s & RS_VAL;
          if (s & RS_INC) break;
          --j;
        }
        st_agent(my, ep | RS_INC | (excl + tot));
      }
    }
    s_gbase[d] = d < nbins ? dbase[d] + excl : 0;
  }
  __syncthreads();
  // stage in digit order
#pragma unroll
  for (int i = 0; i < RS_ITEMS; ++i) {
    const uint64_t idx = wbase + (uint64_t)i * kWave + lane;
    if (idx < n) {
      const uint32_t dd = dig(key[i], s_spl);
      const uint32_t pos = s_tex[dd] + s_wcnt[wave][dd] + rank[i];
      s_keys[pos] = key[i];
      if constexpr (PAIRS) s_vals[pos] = val[i];
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
      const uint32_t dd = dig(k, s_spl);
      const uint64_t o = s_gbase[dd] + (j - s_tex[dd]);
      out[o] = LAST ? (k ^ flip) : k;
      if constexpr (PAIRS) vout[o] = s_vals[j];
    }
  }
}

// sort keys of nut_sort_pairs in unsigned order: int64 with the sign bit flipped, f64 by
// the IEEE total order (-0 < +0, NaNs at the ends); DESC: the complement
__global__ void sort_key_kernel(const uint64_t *__restrict__ in, int type, int desc, uint64_t n,
                                uint64_t *__restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = in[i];
    uint64_t u = type == NUT_T_F64 ? f64_to_ord(b) : (b ^ RS_FLIP);
    out[i] = desc ? ~u : u;
  }
}

// f64 bit patterns <-> int64 words whose signed order is the IEEE total order (-NaN < -inf
// < ... < -0 < +0 < ... < +inf < +NaN): a set sign bit flips the other 63 bits.  The map
// is its own inverse, so the same launch maps the sorted words back.  `canon` (GROUP BY
// keys): -0.0 is +0.0 and every NaN the quiet +NaN first, so equal values share one word.
__global__ void f64_signed_order_kernel(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t n,
                                        int canon) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t b = in[i];
    if (canon) {
      if ((b << 1) == 0) b = 0;                                           // -0.0 -> +0.0
      if ((b & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull) b = kF64CanonNaN;  // NaN -> +qNaN
    }
    out[i] = b ^ ((uint64_t)((int64_t)b >> 63) >> 1);
  }
}

nut_status f64_signed_order(nut_ctx *c, const uint64_t *in, uint64_t *out, uint64_t n, bool canon) {
  if (n == 0) return NUT_OK;
  DeviceGuard g(c->device);
  const unsigned gk = (unsigned)std::min<uint64_t>((n + 255) / 256, (uint64_t)c->num_cus * 16);
  hipLaunchKernelGGL(f64_signed_order_kernel, dim3(gk), dim3(256), 0, c->stream, in, out, n, canon ? 1 : 0);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

// Status granules for `ntiles` tiles, tagged with a fresh pass epoch.  The array is
// cleared only when it is (re)allocated or the 8-bit epoch wraps.
nut_status next_status(nut_ctx *c, uint64_t ntiles, uint64_t **status, uint32_t *epoch) {
  const size_t need = ntiles * RS_BINS * 8;
  nut_status s = c->sort_status.reserve(need);
  if (s) return s;
  if (c->sort_status.ptr != c->sort_status_seen || need > c->sort_status_clean || c->sort_epoch >= 255) {
    NUT_HIP(hipMemsetAsync(c->sort_status.ptr, 0, c->sort_status.bytes, c->stream));
    c->sort_status_seen = c->sort_status.ptr;
    c->sort_status_clean = c->sort_status.bytes;
    c->sort_epoch = 0;
  }
  *epoch = ++c->sort_epoch;
  *status = (uint64_t *)c->sort_status.ptr;
  return NUT_OK;
}

}  // namespace nut

using namespace nut;

// Stable sort of (key, payload) pairs: ORDER BY keys with projected columns.  Keys are
// mapped to unsigned order once (sort_key_kernel), then LSD passes move key and payload
// together; only the permuted payload is returned (the caller gathers its columns
// through it).  16 B/key per executed pass + 8 B/key histogram + 16 B/key key mapping.
extern "C" nut_status nut_sort_pairs(nut_ctx *c, const void *keys, int key_type, int desc, const int64_t *vals,
                                     int64_t *vals_out, uint64_t n) {
  if (!c || (n && (!keys || !vals_out))) return fail(NUT_ERR_INVALID_ARG, "nut_sort_pairs: NULL argument");
  if (key_type != NUT_T_I64 && key_type != NUT_T_F64) return fail(NUT_ERR_INVALID_ARG, "nut_sort_pairs: key type");
  if (n == 0) return NUT_OK;
  DeviceGuard g(c->device);
  const uint64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  if (ntiles > 0x7FFFFFF0ull || n > RS_VAL) return fail(NUT_ERR_UNSUPPORTED, "nut_sort_pairs: n too large");
  hipStream_t st = c->stream;
  // scratch: [err | tickets | hist 8x256 | base 8x256 | trivial] + keys A, keys B, payload B
  const size_t o_hist = 256;
  const size_t o_base = o_hist + 8 * RS_BINS * 8;
  const size_t o_triv = o_base + 8 * RS_BINS * 8;
  const size_t o_ka = (o_triv + 64 + 255) & ~size_t(255);
  const size_t o_kb = o_ka + ((n * 8 + 255) & ~size_t(255));
  const size_t o_vb = o_kb + ((n * 8 + 255) & ~size_t(255));
  nut_status s = c->sort_tmp.reserve(o_vb + n * 8);
  if (s) return s;
  char *b = (char *)c->sort_tmp.ptr;
  uint32_t *err = (uint32_t *)b;
  uint32_t *tickets = (uint32_t *)(b + 16);
  unsigned long long *hist = (unsigned long long *)(b + o_hist);
  uint64_t *base = (uint64_t *)(b + o_base);
  uint32_t *triv = (uint32_t *)(b + o_triv);
  uint64_t *ka = (uint64_t *)(b + o_ka), *kb = (uint64_t *)(b + o_kb), *vb = (uint64_t *)(b + o_vb);
  c->timer.begin(st, NUT_KERNEL_SORT);
  const unsigned gk = (unsigned)std::min<uint64_t>((n + 255) / 256, (uint64_t)c->num_cus * 16);
  hipLaunchKernelGGL(sort_key_kernel, dim3(gk), dim3(256), 0, st, (const uint64_t *)keys, key_type, desc, n, ka);
  NUT_HIP(hipMemsetAsync(b, 0, o_base, st));
  const uint64_t hblocks =
      std::min<uint64_t>((n + 2 * RS_HIST_THREADS - 1) / (2 * RS_HIST_THREADS), (uint64_t)c->num_cus * 4);
  hipLaunchKernelGGL(rs_hist_kernel, dim3((unsigned)hblocks), dim3(RS_HIST_THREADS), 0, st, (const int64_t *)ka, n,
                     (uint64_t)0, hist);
  hipLaunchKernelGGL(rs_scan_kernel, dim3(8), dim3(RS_BINS), 0, st, (const unsigned long long *)hist, n, base, triv);
  NUT_HIP(hipGetLastError());
  uint32_t htriv[8];
  NUT_HIP(hipMemcpyAsync(htriv, triv, sizeof(htriv), hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  int passes[8], np = 0;
  for (int p = 0; p < 8; ++p)
    if (!htriv[p]) passes[np++] = p;
  if (np == 0) passes[np++] = 0;  // all keys equal: one (identity) pass still writes the payload
  c->sort_bytes = 16 * n + 8 * n + 16 * n * (uint64_t)np;
  c->sort_levels = (uint32_t)np;
  // payload ping-pong so that the last pass writes vals_out; keys alternate A / B
  const uint64_t *kin = ka, *vin = (const uint64_t *)vals;
  for (int k = 0; k < np; ++k) {
    uint64_t *kout = (k % 2 == 0) ? kb : ka;
    uint64_t *vout = ((np - 1 - k) % 2 == 0) ? (uint64_t *)vals_out : vb;
    uint64_t *status;
    uint32_t epoch;
    s = next_status(c, ntiles, &status, &epoch);
    if (s) return s;
    const int p = passes[k];
    auto kern = k == 0 ? rs_pass_kernel<true, false, RadixDigit, true> : rs_pass_kernel<false, false, RadixDigit, true>;
    hipLaunchKernelGGL(kern, dim3((unsigned)ntiles), dim3(RS_THREADS), 0, st, (const uint64_t *)kin, kout, n,
                       RadixDigit{8 * p}, (const int64_t *)nullptr, RS_BINS, (uint64_t)0,
                       (const uint64_t *)(base + p * RS_BINS), status, epoch, tickets + k, err,
                       k == 0 ? (const uint64_t *)vals : vin, vout);
    NUT_HIP(hipGetLastError());
    kin = kout;
    vin = vout;
  }
  c->timer.end(st);
  NUT_HIP(hipMemcpyAsync(htriv, err, 4, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  if (htriv[0]) return fail(NUT_ERR_TIMEOUT, "nut_sort_pairs: look-back spin limit hit");
  return NUT_OK;
}

// keys-only sorts run the hybrid MSD radix sort (msd_sort.hip); the LSD passes above
// serve the stable (key, payload) sorts and the sample sort's partition
static nut_status sort_i64(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n, uint64_t flip) {
  if (!c || (n && (!in || !out))) return fail(NUT_ERR_INVALID_ARG, "nut_sort_i64: NULL argument");
  if (n && (uintptr_t)in == (uintptr_t)out) return fail(NUT_ERR_INVALID_ARG, "nut_sort_i64: in and out alias");
  if (n == 0) return NUT_OK;
  DeviceGuard g(c->device);
  return msd_sort_i64(c, in, out, n, flip);
}

extern "C" nut_status nut_sort_i64(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n) {
  return sort_i64(c, in, out, n, RS_FLIP);
}

extern "C" nut_status nut_sort_i64_desc(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n) {
  return sort_i64(c, in, out, n, RS_FLIP_DESC);
}

extern "C" nut_status nut_partition_i64(nut_ctx *c, const int64_t *in, uint64_t n, const int64_t *splitters_host,
                                        int nsplit, int64_t *out, uint64_t *counts_host) {
  if (!c || !counts_host || (n && (!in || !out)) || (nsplit && !splitters_host))
    return fail(NUT_ERR_INVALID_ARG, "nut_partition_i64: NULL argument");
  if (nsplit < 0 || nsplit >= RS_MAX_BUCKETS)
    return fail(NUT_ERR_INVALID_ARG, "nut_partition_i64: 0 <= nsplit < 64 required");
  for (int i = 1; i < nsplit; ++i)
    if (splitters_host[i] < splitters_host[i - 1])
      return fail(NUT_ERR_INVALID_ARG, "nut_partition_i64: splitters must be ascending");
  if (n && (uintptr_t)in == (uintptr_t)out) return fail(NUT_ERR_INVALID_ARG, "nut_partition_i64: in and out alias");
  const int nb = nsplit + 1;
  for (int i = 0; i < nb; ++i) counts_host[i] = 0;
  if (n == 0) return NUT_OK;
  DeviceGuard g(c->device);
  const uint64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  if (ntiles > 0x7FFFFFF0ull || n > RS_VAL) return fail(NUT_ERR_UNSUPPORTED, "nut_partition_i64: n too large");
  // misc scratch: [err 4, ticket 4, pad 8 | hist 64*8 | splitters 64*8 | base 64*8]
  nut_status s = c->misc.reserve(16 + 3 * RS_MAX_BUCKETS * 8 + 64);
  if (s) return s;
  char *b = (char *)c->misc.ptr;
  uint32_t *err = (uint32_t *)b;
  uint32_t *ticket = err + 1;
  unsigned long long *hist = (unsigned long long *)(b + 16);
  int64_t *spl = (int64_t *)(b + 16 + RS_MAX_BUCKETS * 8);
  uint64_t *base = (uint64_t *)(b + 16 + 2 * RS_MAX_BUCKETS * 8);
  hipStream_t st = c->stream;
  BucketDigit dig{nsplit};
  c->timer.begin(st, NUT_KERNEL_SORT);
  NUT_HIP(hipMemsetAsync(b, 0, 16 + RS_MAX_BUCKETS * 8, st));
  if (nsplit) NUT_HIP(hipMemcpyAsync(spl, splitters_host, nsplit * 8, hipMemcpyHostToDevice, st));
  uint64_t hblocks = std::min<uint64_t>((n + RS_HIST_THREADS - 1) / RS_HIST_THREADS, (uint64_t)c->num_cus * 4);
  hipLaunchKernelGGL(pt_hist_kernel, dim3((unsigned)hblocks), dim3(RS_HIST_THREADS), 0, st, in, n, dig,
                     (const int64_t *)spl, hist);
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipMemcpyAsync(counts_host, hist, nb * 8, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  uint64_t hbase[RS_MAX_BUCKETS], run = 0;
  for (int i = 0; i < nb; ++i) {
    hbase[i] = run;
    run += counts_host[i];
  }
  NUT_HIP(hipMemcpyAsync(base, hbase, nb * 8, hipMemcpyHostToDevice, st));
  uint64_t *status;
  uint32_t epoch;
  s = next_status(c, ntiles, &status, &epoch);
  if (s) return s;
  hipLaunchKernelGGL((rs_pass_kernel<false, false, BucketDigit>), dim3((unsigned)ntiles), dim3(RS_THREADS), 0, st,
                     (const uint64_t *)in, (uint64_t *)out, n, dig, (const int64_t *)spl, nb, (uint64_t)0,
                     (const uint64_t *)base, status, epoch, ticket, err, (const uint64_t *)nullptr,
                     (uint64_t *)nullptr);
  NUT_HIP(hipGetLastError());
  c->timer.end(st);
  uint32_t herr = 0;
  NUT_HIP(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  if (herr) return fail(NUT_ERR_TIMEOUT, "nut_partition_i64: look-back spin limit hit");
  return NUT_OK;
}
