// api.hip — context lifecycle, error reporting and the synthetic column source.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <thread>

#include "common.hpp"

namespace nut {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

nut_status fail(nut_status st, const std::string &msg) {
  g_last_error = msg;
  return st;
}

nut_status hip_fail(hipError_t e, const char *what) {
  g_last_error = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
  return e == hipErrorOutOfMemory ? NUT_ERR_OOM : NUT_ERR_HIP;
}

nut_status Scratch::reserve(size_t need, bool grow) {
  if (need <= bytes) return NUT_OK;
  if (ptr) (void)hipFree(ptr);
  ptr = nullptr;
  bytes = 0;
  size_t want = grow ? need + need / 4 : need;
  hipError_t e = hipMalloc(&ptr, want);
  if (e != hipSuccess) {
    ptr = nullptr;
    return hip_fail(e, "hipMalloc(scratch)");
  }
  bytes = want;
  return NUT_OK;
}

void Scratch::release() {
  if (ptr) (void)hipFree(ptr);
  ptr = nullptr;
  bytes = 0;
}

// ------------------------------------------------------------ kernel timer
hipEvent_t KernelTimer::get() {
  if (!pool.empty()) {
    hipEvent_t e = pool.back();
    pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

void KernelTimer::begin(hipStream_t s, int kind) {
  if (!enabled) return;
  Pair p{get(), get(), kind};
  if (p.a) (void)hipEventRecord(p.a, s);
  pending.push_back(p);
}

void KernelTimer::end(hipStream_t s) {
  if (!enabled || pending.empty()) return;
  if (pending.back().b) (void)hipEventRecord(pending.back().b, s);
}

nut_status KernelTimer::drain() {
  for (auto &p : pending) {
    if (p.a && p.b) {
      NUT_HIP(hipEventSynchronize(p.b));
      float ms = 0.f;
      NUT_HIP(hipEventElapsedTime(&ms, p.a, p.b));
      total_ms[p.kind] += ms;
      launches[p.kind] += 1;
    }
    if (p.a) pool.push_back(p.a);
    if (p.b) pool.push_back(p.b);
  }
  pending.clear();
  return NUT_OK;
}

void KernelTimer::release() {
  (void)drain();
  for (auto e : pool) (void)hipEventDestroy(e);
  pool.clear();
}

// ------------------------------------------------------------ generator kernel
__global__ void gen_column_kernel(int kind, uint64_t seed, int64_t a, int64_t b, double c,
                                  uint64_t row0, uint64_t n, void *out) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  int64_t *oi = (int64_t *)out;
  double *od = (double *)out;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t u = gen_u64(seed, row0 + i);
    switch (kind) {
      case NUT_GEN_U62: oi[i] = (int64_t)(u >> 2); break;
      case NUT_GEN_FULL_I64: oi[i] = (int64_t)u; break;
      case NUT_GEN_POOL_KEY: oi[i] = (int64_t)mix64((u % (uint64_t)a) ^ kPoolSalt); break;
      case NUT_GEN_DYADIC: od[i] = (double)(u >> 44) / 64.0; break;
      case NUT_GEN_UNIT_F64: od[i] = (double)(u >> 11) * 0x1p-53; break;
      case NUT_GEN_RANGE_I64: oi[i] = a + (int64_t)(u % (uint64_t)b); break;
      case NUT_GEN_SKEW_KEY: oi[i] = (int64_t)mix64(((u % (uint64_t)a) >> (((mix64(u) >> 59) * 3) >> 2)) ^ kPoolSalt); break;
      default: od[i] = (double)(a + (int64_t)(u % (uint64_t)b)) / c; break;
    }
  }
}

// ------------------------------------------------------------ copy-floor probe
// 16-B chunk i of the read stream is stored when its lane (i mod 64) is below q64: every
// wave-instruction of loads is one contiguous KiB and its stores one contiguous run of
// q64 x 16 B, so reads and writes interleave at the q64 / 64 ratio through the whole pass.
// Four loads in flight per lane; what is not stored folds into a word that is written only
// on an impossible value (keeps the loads live).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_probe_kernel(const u32x4 *__restrict__ src, uint64_t nchunks,
                                                           u32x4 *__restrict__ dst, uint32_t q64,
                                                           u32x4 *__restrict__ sink) {
  constexpr int U = 4;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; base < nchunks; base += stride * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + u * stride;
      if (i < nchunks) v[u] = __builtin_nontemporal_load(src + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + u * stride;
      if (i >= nchunks) break;
      const uint32_t lane = (uint32_t)(i & 63);
      if (lane < q64)
        __builtin_nontemporal_store(v[u], dst + (i >> 6) * q64 + lane);
      else
        acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x] = u32x4{acc, 0u, 0u, 0u};
}

// ------------------------------------------------------------ large D2H
constexpr int kCopyThreads = 8;

nut_status copy_to_host(nut_ctx *c, void *dst, const void *src, size_t bytes) {
  // pinned (page-locked) destination: the copy engine writes it directly at the link rate
  hipPointerAttribute_t pa;
  bool pinned = false;
  if (hipPointerGetAttributes(&pa, dst) == hipSuccess) pinned = pa.type == hipMemoryTypeHost;
  (void)hipGetLastError();  // pageable memory reports an error here
  if (bytes < (8u << 20) || pinned) {  // small or pinned: one plain copy
    NUT_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    NUT_HIP(hipStreamSynchronize(c->stream));
    return NUT_OK;
  }
  for (auto &b : c->stage)
    if (!b) NUT_HIP(hipHostMalloc((void **)&b, kStageBytes, hipHostMallocDefault));
  hipEvent_t ev[2] = {nullptr, nullptr};
  for (auto &e : ev) NUT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const size_t nch = (bytes + kStageBytes - 1) / kStageBytes;
  auto chunk = [&](size_t i) { return std::min(kStageBytes, bytes - i * kStageBytes); };
  hipError_t e = hipMemcpyAsync(c->stage[0], src, chunk(0), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipEventRecord(ev[0], c->stream);
  for (size_t i = 0; i < nch && e == hipSuccess; ++i) {
    if (i + 1 < nch) {  // the next chunk's transfer overlaps this chunk's host copy
      e = hipMemcpyAsync(c->stage[(i + 1) & 1], (const char *)src + (i + 1) * kStageBytes, chunk(i + 1),
                         hipMemcpyDeviceToHost, c->stream);
      if (e == hipSuccess) e = hipEventRecord(ev[(i + 1) & 1], c->stream);
    }
    if (e == hipSuccess) e = hipEventSynchronize(ev[i & 1]);
    if (e != hipSuccess) break;
    const char *from = c->stage[i & 1];
    char *to = (char *)dst + i * kStageBytes;
    const size_t len = chunk(i), per = (len + kCopyThreads - 1) / kCopyThreads;
    std::thread th[kCopyThreads];
    for (int t = 0; t < kCopyThreads; ++t) {
      const size_t a = std::min(len, t * per), b = std::min(len, a + per);
      th[t] = std::thread([=] { memcpy(to + a, from + a, b - a); });
    }
    for (auto &t : th) t.join();
  }
  // the staging buffer of the last chunk must not be rewritten before its event
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  for (auto &ev1 : ev) (void)hipEventDestroy(ev1);
  return e == hipSuccess ? NUT_OK : hip_fail(e, "copy_to_host");
}

}  // namespace nut

using namespace nut;

extern "C" {

int nut_abi_version(void) { return NUTEXEC_ABI_VERSION; }

const char *nut_last_error(void) { return g_last_error.c_str(); }

nut_status nut_ctx_create(int device, nut_ctx **out) {
  if (!out) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_create: out is NULL");
  *out = nullptr;
  int ndev = 0;
  NUT_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return fail(NUT_ERR_INVALID_ARG, "nut_ctx_create: device " + std::to_string(device) +
                                         " out of range (" + std::to_string(ndev) + " devices)");
  DeviceGuard g(device);
  hipDeviceProp_t prop;
  NUT_HIP(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(NUT_ERR_UNSUPPORTED, std::string("nutexec is built for gfx950 (MI355X); device is ") +
                                         prop.gcnArchName);
  nut_ctx *c = new nut_ctx();
  c->device = device;
  c->num_cus = prop.multiProcessorCount;
  snprintf(c->name, sizeof(c->name), "%s", prop.name);
  hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return hip_fail(e, "hipStreamCreate");
  }
  c->stream = c->own_stream;
  {  // the device's stream-ordered pool keeps what queries free (hipMallocAsync scratch,
     // sql_plan.cpp DevBuf) instead of returning it at every synchronisation
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
      uint64_t keep = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
    (void)hipGetLastError();
  }
  e = hipHostMalloc((void **)&c->host_pinned, 4096, hipHostMallocDefault);
  if (e != hipSuccess) {
    (void)hipStreamDestroy(c->own_stream);
    delete c;
    return hip_fail(e, "hipHostMalloc");
  }
  *out = c;
  return NUT_OK;
}

}  // extern "C"

namespace nut {

nut_status pool_take(nut_ctx *c, size_t bytes, void **p, size_t *got) {
  if (c->tbl_pool && c->tbl_pool_bytes >= bytes) {
    *p = c->tbl_pool;
    *got = c->tbl_pool_bytes;
    c->tbl_pool = nullptr;
    c->tbl_pool_bytes = 0;
    return NUT_OK;
  }
  NUT_HIP(hipMalloc(p, bytes));
  *got = bytes;
  return NUT_OK;
}

void pool_give(nut_ctx *c, void *p, size_t bytes) {
  if (!p) return;
  DeviceGuard dg(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (bytes >= c->tbl_pool_bytes) {
    if (c->tbl_pool) (void)hipFree(c->tbl_pool);
    c->tbl_pool = p;
    c->tbl_pool_bytes = bytes;
  } else {
    (void)hipFree(p);
  }
}

}  // namespace nut

extern "C" {

void nut_ctx_destroy(nut_ctx *c) {
  if (!c) return;
  DeviceGuard g(c->device);
  (void)hipStreamSynchronize(c->stream);
  c->filter_state.release();
  c->sort_tmp.release();
  c->sort_tmp2.release();
  c->sort_status.release();
  c->sort_meta.release();
  c->gp_data.release();
  c->gp_meta.release();
  c->misc.release();
  c->timer.release();
  for (auto &b : c->stage)
    if (b) (void)hipHostFree(b);
  if (c->tbl_pool) (void)hipFree(c->tbl_pool);
  if (c->host_pinned) (void)hipHostFree(c->host_pinned);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->aux_stream) (void)hipStreamDestroy(c->aux_stream);
  if (c->order_stream) (void)hipStreamDestroy(c->order_stream);
  delete c;
}

nut_status nut_ctx_set_stream(nut_ctx *c, void *s) {
  if (!c) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_set_stream: ctx is NULL");
  c->stream = (hipStream_t)s;  // NULL is the device's default (null) stream, a valid target
  return NUT_OK;
}

nut_status nut_ctx_sync(nut_ctx *c) {
  if (!c) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_sync: ctx is NULL");
  DeviceGuard g(c->device);
  NUT_HIP(hipStreamSynchronize(c->stream));
  return NUT_OK;
}

nut_status nut_ctx_memcpy(nut_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c || (bytes && (!dst || !src))) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_memcpy: NULL argument");
  if (bytes == 0) return NUT_OK;
  DeviceGuard g(c->device);
  NUT_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  return NUT_OK;
}

nut_status nut_ctx_enable_timing(nut_ctx *c, int enable) {
  if (!c) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_enable_timing: ctx is NULL");
  DeviceGuard g(c->device);
  nut_status st = c->timer.drain();
  c->timer.enabled = enable != 0;
  for (int k = 0; k < 4; ++k) c->timer.total_ms[k] = 0, c->timer.launches[k] = 0;
  return st;
}

nut_status nut_ctx_sort_stats(nut_ctx *c, uint64_t *bytes, uint32_t *levels) {
  if (!c) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_sort_stats: NULL context");
  if (bytes) *bytes = c->sort_bytes;
  if (levels) *levels = c->sort_levels;
  return NUT_OK;
}

nut_status nut_ctx_groupby_stats(nut_ctx *c, uint32_t *path, uint32_t *levels, uint32_t *optimistic) {
  if (!c) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_groupby_stats: NULL context");
  if (path) *path = c->gb_path;
  if (levels) *levels = c->gb_levels;
  if (optimistic) *optimistic = c->gb_optimistic;
  return NUT_OK;
}

nut_status nut_ctx_set_option(nut_ctx *c, int option, int64_t value) {
  if (!c || option < 0 || option >= NUT_OPT_COUNT) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_set_option: bad option");
  static const int64_t lo[NUT_OPT_COUNT] = {-1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 6, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 512, 2, 0},
                       hi[NUT_OPT_COUNT] = {1, 2, 1, 1, 64, 1, 4, 4, 8, 1, 8, 1, 8, 32, 256, 16, 16, 16, 1024, 1, 1, 2, 1, 1024, 8, 128};
  if (value < lo[option] || value > hi[option])
    return fail(NUT_ERR_INVALID_ARG, "nut_ctx_set_option: value " + std::to_string(value) + " out of range [" +
                                         std::to_string(lo[option]) + ", " + std::to_string(hi[option]) + "]");
  if (option == NUT_OPT_PRIV_BD && value && value != 128 && value != 192 && value != 256)
    return fail(NUT_ERR_INVALID_ARG, "nut_ctx_set_option: NUT_OPT_PRIV_BD takes 0, 128, 192 or 256");
  if (option == NUT_OPT_SORT_BD && value && value != 512 && value != 1024)
    return fail(NUT_ERR_INVALID_ARG, "nut_ctx_set_option: NUT_OPT_SORT_BD takes 0, 512 or 1024");
  if (option == NUT_OPT_GB_L1_THREADS && value != 512 && value != 1024)
    return fail(NUT_ERR_INVALID_ARG, "nut_ctx_set_option: NUT_OPT_GB_L1_THREADS takes 512 or 1024");
  c->opt[option] = value;
  return NUT_OK;
}

nut_status nut_ctx_get_option(nut_ctx *c, int option, int64_t *value) {
  if (!c || !value || option < 0 || option >= NUT_OPT_COUNT)
    return fail(NUT_ERR_INVALID_ARG, "nut_ctx_get_option: bad argument");
  *value = c->opt[option];
  return NUT_OK;
}

nut_status nut_ctx_kernel_time(nut_ctx *c, int kind, double *total_ms, uint64_t *launches) {
  if (!c || kind < 0 || kind > 3) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_kernel_time: bad argument");
  DeviceGuard g(c->device);
  nut_status st = c->timer.drain();
  if (st) return st;
  if (total_ms) *total_ms = c->timer.total_ms[kind];
  if (launches) *launches = c->timer.launches[kind];
  c->timer.total_ms[kind] = 0;
  c->timer.launches[kind] = 0;
  return NUT_OK;
}

nut_status nut_ctx_info(nut_ctx *c, int *num_cus, char *name, size_t name_len) {
  if (!c) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_info: ctx is NULL");
  if (num_cus) *num_cus = c->num_cus;
  if (name && name_len) snprintf(name, name_len, "%s", c->name);
  return NUT_OK;
}

nut_status nut_stream_probe(nut_ctx *c, const void *src, uint64_t read_bytes, void *dst, uint64_t write_bytes,
                            int reps, double *best_ms) {
  if (!c || !best_ms || reps < 1 || !src || read_bytes == 0 || (write_bytes && !dst) || write_bytes > read_bytes ||
      (read_bytes | write_bytes | (uintptr_t)src | (uintptr_t)dst) % 16)
    return fail(NUT_ERR_INVALID_ARG, "nut_stream_probe: bad argument (16-B multiples, write_bytes <= read_bytes)");
  DeviceGuard g(c->device);
  const uint64_t nchunks = read_bytes / 16;
  const uint32_t q64 = (uint32_t)((unsigned __int128)write_bytes * 64 / read_bytes);
  // workgroups per CU: the option, or the best of 2 / 4 / 8 (the fastest occupancy depends on
  // the stream: 2 for a pure read, 8 for the filter's 2:1 read:write mix, measured)
  const unsigned fixed = (unsigned)c->opt[NUT_OPT_STREAM_BLOCKS];
  const unsigned tries[3] = {2, 4, 8};
  if (nut_status st = c->misc.reserve((size_t)c->num_cus * 32 * 16)) return st;
  hipEvent_t ev[2] = {nullptr, nullptr};
  for (auto &e : ev) NUT_HIP(hipEventCreate(&e));
  float best = 0.f;
  bool have = false;
  hipError_t e = hipSuccess;
  for (int t = 0; t < (fixed ? 1 : 3) && e == hipSuccess; ++t) {
    const unsigned blocks = (unsigned)c->num_cus * (fixed ? fixed : tries[t]);
    for (int r = 0; r < reps && e == hipSuccess; ++r) {
      e = hipEventRecord(ev[0], c->stream);
      hipLaunchKernelGGL(stream_probe_kernel, dim3(blocks), dim3(256), 0, c->stream, (const u32x4 *)src, nchunks,
                         (u32x4 *)dst, q64, (u32x4 *)c->misc.ptr);
      if (e == hipSuccess) e = hipGetLastError();
      if (e == hipSuccess) e = hipEventRecord(ev[1], c->stream);
      if (e == hipSuccess) e = hipEventSynchronize(ev[1]);
      float ms = 0.f;
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, ev[0], ev[1]);
      if (e == hipSuccess && (!have || ms < best)) best = ms, have = true;
    }
  }
  for (auto &x : ev) (void)hipEventDestroy(x);
  if (e != hipSuccess) return hip_fail(e, "nut_stream_probe");
  *best_ms = best;
  return NUT_OK;
}

nut_status nut_gen_column(nut_ctx *c, int kind, uint64_t seed, int64_t a, int64_t b, double cc,
                          uint64_t row0, uint64_t n, void *out) {
  if (!c || (!out && n)) return fail(NUT_ERR_INVALID_ARG, "nut_gen_column: NULL argument");
  if (kind < NUT_GEN_U62 || kind > NUT_GEN_SKEW_KEY)
    return fail(NUT_ERR_INVALID_ARG, "nut_gen_column: unknown kind " + std::to_string(kind));
  if (((kind == NUT_GEN_POOL_KEY || kind == NUT_GEN_SKEW_KEY) && a <= 0) ||
      ((kind == NUT_GEN_RANGE_I64 || kind == NUT_GEN_RANGE_F64) && b <= 0))
    return fail(NUT_ERR_INVALID_ARG, "nut_gen_column: empty range");
  if (n == 0) return NUT_OK;
  DeviceGuard g(c->device);
  uint64_t blocks = (n + 255) / 256;
  uint64_t cap = (uint64_t)c->num_cus * 16;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(gen_column_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, kind,
                     seed, a, b, cc, row0, n, out);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

}  // extern "C"
