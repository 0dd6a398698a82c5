// topk.hip — ORDER BY ... LIMIT k without sorting every row (LimitClause,
// /root/reference/src/parser/ast/query.rs:92-98; SURVEY.md §8(a) B5's caller).
//
// Radix select on the order-mapped keys (int64: sign bit flipped; f64: IEEE total order;
// DESC: complemented — the map nut_sort_pairs sorts by): 12-bit digit histograms, most
// significant first, each restricted to the keys that share the digits chosen so far,
// until the bucket holding the k-th key leaves few enough candidates; then one pass
// collects the positions of every key ordered at or before that bucket's last value.  The
// candidates (>= k, every tie at the boundary included) are what a stable sort needs to
// produce the first k rows exactly as a full sort would.  HBM: 8 B/key per histogram level
// (one or two at 1e8-1e9 uniform keys) + 8 B/key for the collection, against a full sort's
// 48-136 B/key.
#include "common.hpp"

namespace nut {

constexpr int TK_BITS = 12;
constexpr int TK_BINS = 1 << TK_BITS;
constexpr int TK_THREADS = 256;
constexpr int TK_UNROLL = 4;

__device__ __forceinline__ uint64_t tk_ord(uint64_t b, int type, int desc) {
  const uint64_t u = type == NUT_T_F64 ? f64_to_ord(b) : (b ^ 0x8000000000000000ull);
  return desc ? ~u : u;
}

// histogram of (u >> shift) & mask over the keys with (u >> top) == prefix (top = 64: all)
__global__ __launch_bounds__(TK_THREADS) void topk_hist_kernel(const uint64_t *__restrict__ keys, uint64_t n,
                                                               int type, int desc, uint64_t prefix, int top,
                                                               int shift, uint32_t mask,
                                                               unsigned long long *__restrict__ hist) {
  __shared__ uint32_t h[TK_BINS];
  for (int i = threadIdx.x; i < TK_BINS; i += TK_THREADS) h[i] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * TK_THREADS;
  for (uint64_t i0 = (uint64_t)blockIdx.x * TK_THREADS + threadIdx.x; i0 < n; i0 += stride * TK_UNROLL) {
    uint64_t v[TK_UNROLL];
#pragma unroll
    for (int j = 0; j < TK_UNROLL; ++j) v[j] = __builtin_nontemporal_load(keys + min(i0 + j * stride, n - 1));
#pragma unroll
    for (int j = 0; j < TK_UNROLL; ++j) {
      const uint64_t u = tk_ord(v[j], type, desc);
      if (i0 + j * stride < n && (top >= 64 || (u >> top) == prefix)) atomicAdd(&h[(uint32_t)(u >> shift) & mask], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TK_BINS; i += TK_THREADS)
    if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

// positions i with ord(key[i]) <= bound, in any order (wave-aggregated appends)
__global__ __launch_bounds__(TK_THREADS) void topk_collect_kernel(const uint64_t *__restrict__ keys, uint64_t n,
                                                                  int type, int desc, uint64_t bound,
                                                                  int64_t *__restrict__ pos,
                                                                  unsigned long long *__restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const uint64_t stride = (uint64_t)gridDim.x * TK_THREADS;
  for (uint64_t i0 = (uint64_t)blockIdx.x * TK_THREADS + threadIdx.x; i0 - threadIdx.x % 64 < n; i0 += stride) {
    const bool in = i0 < n && tk_ord(keys[min(i0, n - 1)], type, desc) <= bound;
    const uint64_t m = __ballot(in);
    if (!m) continue;
    const int leader = __builtin_ctzll(m);
    unsigned long long b = 0;
    if (lane == leader) b = atomicAdd(cnt, (unsigned long long)__popcll(m));
    b = __shfl(b, leader, 64);
    if (in) pos[b + lane_rank(m)] = (int64_t)i0;
  }
}

__global__ void topk_iota_kernel(int64_t *__restrict__ out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = (int64_t)i;
}

}  // namespace nut

using namespace nut;

extern "C" nut_status nut_topk_positions(nut_ctx *c, const void *keys, int key_type, int desc, uint64_t n, uint64_t k,
                                         int64_t *positions, uint64_t cap, uint64_t *count_host) {
  if (!c || !count_host || (n && !keys)) return fail(NUT_ERR_INVALID_ARG, "nut_topk_positions: NULL argument");
  if (key_type != NUT_T_I64 && key_type != NUT_T_F64) return fail(NUT_ERR_INVALID_ARG, "nut_topk_positions: key type");
  *count_host = 0;
  if (n == 0 || k == 0) return NUT_OK;
  DeviceGuard g(c->device);
  hipStream_t st = c->stream;
  if (k >= n) {  // every key
    *count_host = n;
    if (n > cap) return NUT_ERR_CAPACITY;
    if (!positions) {
    c->timer.end(st);
    return fail(NUT_ERR_INVALID_ARG, "nut_topk_positions: NULL output");
  }
    hipLaunchKernelGGL(topk_iota_kernel, dim3((unsigned)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256), 0, st,
                       positions, n);
    NUT_HIP(hipGetLastError());
    return NUT_OK;
  }
  nut_status s = c->misc.reserve(TK_BINS * 8 + 64);
  if (s) return s;
  unsigned long long *dhist = (unsigned long long *)c->misc.ptr;
  unsigned long long *dcnt = dhist + TK_BINS;
  std::vector<unsigned long long> h(TK_BINS);
  const unsigned grid = (unsigned)std::min<uint64_t>((n + TK_THREADS * TK_UNROLL - 1) / (TK_THREADS * TK_UNROLL),
                                                     (uint64_t)c->num_cus * 8);
  // stop once the candidates are few: a stable sort of them is then cheap
  const uint64_t stop = std::max<uint64_t>(4 * k, 1ull << 16);
  uint64_t prefix = 0, below = 0, cand = n, bound = ~0ull;
  int top = 64;
  c->timer.begin(st, NUT_KERNEL_SORT);
  for (;;) {
    const int shift = std::max(0, top - TK_BITS);
    const uint32_t mask = (uint32_t)((1ull << (top - shift)) - 1);
    NUT_HIP(hipMemsetAsync(dhist, 0, TK_BINS * 8, st));
    hipLaunchKernelGGL(topk_hist_kernel, dim3(grid), dim3(TK_THREADS), 0, st, (const uint64_t *)keys, n, key_type,
                       desc, prefix, top, shift, mask, dhist);
    NUT_HIP(hipGetLastError());
    NUT_HIP(hipMemcpyAsync(h.data(), dhist, TK_BINS * 8, hipMemcpyDeviceToHost, st));
    NUT_HIP(hipStreamSynchronize(st));
    uint32_t b = 0;
    while (b < mask && below + h[b] < k) below += h[b++];
    cand = below + h[b];
    prefix = (top >= 64 ? 0 : prefix << (top - shift)) | b;
    top = shift;
    if (cand <= stop || shift == 0) {
      bound = shift ? (prefix << shift) | ((1ull << shift) - 1) : prefix;
      break;
    }
  }
  *count_host = cand;
  if (cand > cap) {
    c->timer.end(st);
    return NUT_ERR_CAPACITY;
  }
  if (!positions) {
    c->timer.end(st);
    return fail(NUT_ERR_INVALID_ARG, "nut_topk_positions: NULL output");
  }
  // collect (unordered) into scratch, then sort the positions ascending into `positions`
  int64_t *tmp = nullptr;
  NUT_HIP(hipMallocAsync((void **)&tmp, cand * 8, st));
  NUT_HIP(hipMemsetAsync(dcnt, 0, 8, st));
  const unsigned gc = (unsigned)std::min<uint64_t>((n + TK_THREADS - 1) / TK_THREADS, (uint64_t)c->num_cus * 16);
  hipLaunchKernelGGL(topk_collect_kernel, dim3(gc), dim3(TK_THREADS), 0, st, (const uint64_t *)keys, n, key_type, desc,
                     bound, tmp, dcnt);
  NUT_HIP(hipGetLastError());
  c->timer.end(st);
  s = nut_sort_i64(c, tmp, positions, cand);
  (void)hipFreeAsync(tmp, st);
  return s;
}
