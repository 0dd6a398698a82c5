// common.hpp — device helpers and host-side context shared by the nutexec kernels.
// MI355X (gfx950, CDNA4) only: wave64, 256 CUs in 8 XCDs, 160 KiB LDS per CU.
#pragma once

#ifndef __HIPCC_RTC__  // also compiled at run time by hipRTC (jit.cpp): device part only
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>
#endif

#include "nutexec.h"

namespace nut {

// ---------------------------------------------------------------- constants
constexpr int kWave = 64;
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kPoolSalt = 0x5DEECE66D2545F49ull;
constexpr uint64_t kEmpty = 0x8000000000000000ull;  // hash-table empty fingerprint

// ---------------------------------------------------------------- hashing
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t gen_u64(uint64_t seed, uint64_t row) {
  return mix64(seed + (row + 1) * kGolden);
}
// owner rank of a group for the multi-GPU exchange
__host__ __device__ __forceinline__ uint64_t owner_hash(uint64_t k1, uint64_t k2, int nk) {
  uint64_t h = mix64(k1 ^ 0x6A09E667F3BCC908ull);
  if (nk == 2) h = mix64(h ^ k2);
  return h;
}
// 2-key fingerprint (not injective: the table verifies the tuple)
__device__ __forceinline__ uint64_t fp2(uint64_t k1, uint64_t k2) {
  uint64_t f = mix64(k1 ^ mix64(k2 + kGolden));
  return f == kEmpty ? (kEmpty ^ 1ull) : f;
}
// multiply-shift slot index
__device__ __forceinline__ uint32_t slot_of(uint64_t fp, int log2cap) {
  return (uint32_t)((fp * kGolden) >> (64 - log2cap));
}

// IEEE total order on f64 bit patterns, mapped to an unsigned integer order
__host__ __device__ __forceinline__ uint64_t f64_to_ord(uint64_t b) {
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__host__ __device__ __forceinline__ uint64_t ord_to_f64(uint64_t o) {
  return (o >> 63) ? (o & 0x7FFFFFFFFFFFFFFFull) : ~o;
}

__device__ __forceinline__ double as_f64(uint64_t b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ uint64_t as_u64(double d) { return (uint64_t)__double_as_longlong(d); }

// number of set bits of `mask` below this lane (v_mbcnt)
__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// relaxed agent-scope atomics (global_load/store ... sc1): single 8-byte granules
__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Coherent read of a word that other workgroups update with memory-side atomics.
// A plain or sc1 load can be served by this XCD's L2 from a line cached before the
// update (measured: a spin on `atomicAdd(p, 0)`, which LLVM folds into a
// `global_load sc1`, never saw another XCD's atomic swap).  A volatile RMW cannot be
// folded and executes at the memory side.  (LLVM folds an idempotent fetch_or/add
// into a load even through a volatile pointer; a compare-exchange whose swap value
// equals its compare value is left alone and returns the current word unchanged.)
__device__ __forceinline__ uint32_t rmw_load(uint32_t *p) {
  return atomicCAS((unsigned int *)p, 0u, 0u);
}
__device__ __forceinline__ uint64_t rmw_load(uint64_t *p) {
  return (uint64_t)atomicCAS((unsigned long long *)p, 0ull, 0ull);
}

__device__ __forceinline__ bool cmp_i64(int64_t v, int op, int64_t k) {
  switch (op) {
    case NUT_LT: return v < k;
    case NUT_LE: return v <= k;
    case NUT_GT: return v > k;
    case NUT_GE: return v >= k;
    case NUT_EQ: return v == k;
    default: return v != k;
  }
}
__device__ __forceinline__ bool cmp_f64(double v, int op, double k) {
  switch (op) {
    case NUT_LT: return v < k;
    case NUT_LE: return v <= k;
    case NUT_GT: return v > k;
    case NUT_GE: return v >= k;
    case NUT_EQ: return v == k;
    default: return v != k;
  }
}

typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

#ifndef __HIPCC_RTC__
// ---------------------------------------------------------------- host side
void set_error(const std::string &msg);
nut_status fail(nut_status st, const std::string &msg);
nut_status hip_fail(hipError_t e, const char *what);

#define NUT_HIP(call)                                  \
  do {                                                 \
    hipError_t e_ = (call);                            \
    if (e_ != hipSuccess) return ::nut::hip_fail(e_, #call); \
  } while (0)

// Multi-GPU merge of partial groups (aggregate.hip, used by dist.cpp): words per group,
// and the spec that folds c partial groups stored column-major at seg (the
// nut_groups_to_device layout of g) into a result of g's shape (SUM and COUNT partials
// add, MIN/MAX re-min/max).  nodes: NUT_MAX_AGGS program nodes the spec may point to.
int groups_width(const nut_groups *g);
void groups_merge_spec(const nut_groups *g, const uint64_t *seg, uint64_t c, nut_agg_spec *s, nut_prog_node *nodes);

// Device -> pageable host copy of a large result, synchronous (api.hip): chunks go
// through two pinned staging buffers while host threads move the previous chunk into
// place — a plain hipMemcpy to pageable (often untouched, freshly allocated) memory ran
// at ~10 GB/s, its page faults and staging copies serialised on one thread.
nut_status copy_to_host(nut_ctx *c, void *dst, const void *src, size_t bytes);
// the context's one cached large allocation (group tables, join tables): pool_take hands it
// out when it holds >= bytes (*got = its size) or hipMallocs exactly `bytes`; pool_give
// syncs the stream and keeps the larger of the returned and the cached allocation
nut_status pool_take(nut_ctx *c, size_t bytes, void **p, size_t *got);
void pool_give(nut_ctx *c, void *p, size_t bytes);

constexpr size_t kStageBytes = 32u << 20;  // nut_ctx::stage: each pinned chunk

// Device scratch that only grows; reused across calls (no malloc in steady state).
struct Scratch {
  void *ptr = nullptr;
  size_t bytes = 0;
  // grow: allocate 25 % more than asked, for buffers whose size creeps up call by call
  nut_status reserve(size_t need, bool grow = true);
  void release();
};

}  // namespace nut

namespace nut {
// hipEvent pairs around hot-kernel launches (only while timing is enabled)
struct KernelTimer {
  struct Pair {
    hipEvent_t a, b;
    int kind;
  };
  bool enabled = false;
  std::vector<Pair> pending;
  std::vector<hipEvent_t> pool;
  double total_ms[4] = {0, 0, 0, 0};
  uint64_t launches[4] = {0, 0, 0, 0};
  hipEvent_t get();
  void begin(hipStream_t s, int kind);
  void end(hipStream_t s);
  nut_status drain();
  void release();
};
}  // namespace nut

struct nut_ctx {
  int device = 0;
  int num_cus = 256;
  char name[64] = {0};
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // device -> host transfers beside the work (nut_groupby_to_host)
  hipStream_t aux_stream = nullptr;   // a second compute stream (nut_groupby_to_host's per-chunk aggregation)
  hipStream_t order_stream = nullptr; //   and a third (its per-chunk ordering, beside the next chunk's aggregation)
  nut::Scratch filter_state;  // tile counter + look-back status words
  nut::Scratch sort_tmp;      // sort ping-pong + histograms
  nut::Scratch sort_tmp2;     // MSD sort, capped layout: the second level's regions
  nut::Scratch sort_status;   // radix-pass look-back granules, epoch-tagged (sort.hip)
  void *sort_status_seen = nullptr;
  size_t sort_status_clean = 0;
  uint32_t sort_epoch = 0;
  uint64_t sort_bytes = 0;   // algorithmic bytes of the last sort (nut_ctx_sort_stats)
  uint32_t sort_levels = 0;
  nut::Scratch sort_meta;     // MSD sort per-level segment / tile / histogram tables (msd_sort.hip)
  nut::Scratch gp_data;       // partitioned aggregation: staged / partitioned records (aggregate.hip)
  nut::Scratch gp_meta;       //   and their per-level tables
  nut::Scratch misc;
  uint64_t *host_pinned = nullptr;  // small pinned staging for counts/flags
  char *stage[2] = {nullptr, nullptr};  // copy_to_host's pinned chunks (allocated on first use)
  void *tbl_pool = nullptr;             // the last freed group table's allocation, for reuse:
  size_t tbl_pool_bytes = 0;            //   hipMalloc / hipFree of a 10^7-group table cost ms
  nut::KernelTimer timer;
  // nut_ctx_set_option (tuning / tests; defaults = the product choice, nut_option order)
  int64_t opt[NUT_OPT_COUNT] = {-1, 0, 1, 1, 8, 1, 0, 0, 2, 1, 6, 1, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1024, 4, 32};
  int priv_probe = -1;  // the compiled Q1 kernel's shape during the shape probe (aggregate.hip)
  uint32_t gb_path = 0, gb_levels = 0, gb_optimistic = 0;  // nut_ctx_groupby_stats
  uint64_t gb_overflow_rows = 0;  // nut_ctx_groupby_overflow (the ordered path's arenas)
  uint32_t gb_heavy_keys = 0;     // nut_ctx_groupby_heavy (the ordered path's heavy-key split)
  uint64_t gb_heavy_rows = 0;
  uint32_t gb_decline = 0;        //   and why the ordered path last declined (nut_gb_decline)
};

namespace nut {
// RAII device guard: switch to ctx->device for the call, restore afterwards.  It also
// clears this thread's HIP last-error slot on entry and exit: other libraries in the
// process (torch, RCCL) leave stale errors there (measured: an ncclAllToAllv left
// hipErrorInvalidDevice), the launch checks below (NUT_HIP(hipGetLastError())) must see
// only this call's errors, and a caller's own checks must not see ours (every error this
// library meets is returned as a status).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    (void)hipGetLastError();
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    (void)hipGetLastError();  // and leaves none behind for the caller's own checks (torch's)
  }
};
}  // namespace nut
#else
}  // namespace nut
#endif  // __HIPCC_RTC__
