// join.hip — hash equi-join on one int64 key.
//
// Build: the build keys are bucketed by the top bits of mix64(key) into a CSR table
// (bucket counts -> exclusive scan -> fill), keys stored in bucket order next to their row
// ids, so a probe scans one short contiguous run (>= 2 buckets per build row: ~0.5 keys per
// bucket).  Probe: a tile of 4096 probe rows counts its output pairs (one bucket scan per
// row), the tile totals are scanned, then the tile re-probes and writes its pairs at its
// offset — pairs come out in probe-row order with no per-row count array in HBM.
#include <algorithm>
#include <vector>

#include "common.hpp"

namespace nut {

constexpr int HJ_THREADS = 256;
constexpr int HJ_ITEMS = 16;
constexpr uint32_t HJ_TILE = HJ_THREADS * HJ_ITEMS;  // probe rows per tile

__device__ __forceinline__ uint64_t hj_bucket(int64_t k, int log2b) {
  return log2b ? mix64((uint64_t)k ^ 0x3C6EF372FE94F82Aull) >> (64 - log2b) : 0;
}

__global__ void hj_count_kernel(const int64_t *__restrict__ keys, uint64_t n, int log2b, uint32_t *__restrict__ cnt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[hj_bucket(keys[i], log2b)], 1u);
}

// exclusive scan of u32 counts into u64 offsets: per-block sums, one-block scan of the sums,
// per-block add (generic helpers for the two scans the join needs)
constexpr int SC_THREADS = 1024;
constexpr int SC_ITEMS = 8;
constexpr uint64_t SC_TILE = SC_THREADS * SC_ITEMS;

template <class T>
__device__ __forceinline__ uint64_t block_scan_excl(uint64_t x, uint64_t *ws, uint64_t *total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint64_t incl = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) ws[wave] = incl;
  __syncthreads();
  uint64_t add = 0, tot = 0;
  for (int w = 0; w < (int)(blockDim.x / kWave); ++w) {
    const uint64_t sw = ws[w];
    add += (w < wave) ? sw : 0;
    tot += sw;
  }
  *total = tot;
  return incl - x + add;
}

template <class T>
__global__ __launch_bounds__(SC_THREADS) void scan_reduce_kernel(const T *__restrict__ in, uint64_t n,
                                                                 uint64_t *__restrict__ sums) {
  __shared__ uint64_t ws[SC_THREADS / kWave];
  const uint64_t base = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_ITEMS;
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < SC_ITEMS; ++i)
    if (base + i < n) x += in[base + i];
  uint64_t tot;
  (void)block_scan_excl<T>(x, ws, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// one block: exclusive scan of `n` sums in place; sums[n] = total
__global__ __launch_bounds__(SC_THREADS) void scan_sums_kernel(uint64_t *__restrict__ sums, uint64_t n) {
  __shared__ uint64_t ws[SC_THREADS / kWave];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t b = 0; b < n; b += SC_THREADS) {
    const uint64_t i = b + threadIdx.x;
    const uint64_t x = i < n ? sums[i] : 0;
    uint64_t tot;
    const uint64_t e = block_scan_excl<uint64_t>(x, ws, &tot);
    const uint64_t c = carry;
    if (i < n) sums[i] = c + e;
    __syncthreads();
    if (threadIdx.x == 0) carry = c + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[n] = carry;
}

template <class T>
__global__ __launch_bounds__(SC_THREADS) void scan_apply_kernel(const T *__restrict__ in, uint64_t n,
                                                                const uint64_t *__restrict__ sums,
                                                                uint64_t *__restrict__ out) {
  __shared__ uint64_t ws[SC_THREADS / kWave];
  const uint64_t base = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_ITEMS;
  T v[SC_ITEMS];
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < SC_ITEMS; ++i) {
    v[i] = base + i < n ? in[base + i] : 0;
    x += v[i];
  }
  uint64_t tot;
  uint64_t run = sums[blockIdx.x] + block_scan_excl<T>(x, ws, &tot);
#pragma unroll
  for (int i = 0; i < SC_ITEMS; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = sums[gridDim.x];
}

__global__ void hj_fill_kernel(const int64_t *__restrict__ keys, uint64_t n, int log2b,
                               unsigned long long *__restrict__ cursor, int64_t *__restrict__ bkeys,
                               int64_t *__restrict__ brow) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t k = keys[i];
    const uint64_t pos = atomicAdd(&cursor[hj_bucket(k, log2b)], 1ull);
    bkeys[pos] = k;
    brow[pos] = (int64_t)i;
  }
}

// output pairs of one probe row
__device__ __forceinline__ uint32_t hj_out_count(uint32_t matches, int type) {
  switch (type) {
    case NUT_JOIN_INNER: return matches;
    case NUT_JOIN_LEFT: return matches ? matches : 1u;
    case NUT_JOIN_SEMI: return matches ? 1u : 0u;
    default: return matches ? 0u : 1u;
  }
}

struct HjTable {
  const uint64_t *off;  // [nbuckets + 1]
  const int64_t *bkeys, *brow;
  int log2b;
};

__device__ __forceinline__ uint32_t hj_matches(const HjTable &t, int64_t k, uint64_t &lo, uint64_t &hi) {
  const uint64_t b = hj_bucket(k, t.log2b);
  lo = t.off[b];
  hi = t.off[b + 1];
  uint32_t m = 0;
  for (uint64_t j = lo; j < hi; ++j) m += t.bkeys[j] == k;
  return m;
}

// pass 1: output pairs per probe tile
__global__ __launch_bounds__(HJ_THREADS) void hj_probe_count_kernel(HjTable t, const int64_t *__restrict__ probe,
                                                                    uint64_t n, int type,
                                                                    uint64_t *__restrict__ tile_cnt) {
  __shared__ uint64_t ws[HJ_THREADS / kWave];
  const uint64_t base = (uint64_t)blockIdx.x * HJ_TILE + threadIdx.x;
  uint64_t c = 0;
#pragma unroll 4
  for (int i = 0; i < HJ_ITEMS; ++i) {
    const uint64_t r = base + (uint64_t)i * HJ_THREADS;
    if (r < n) {
      uint64_t lo, hi;
      c += hj_out_count(hj_matches(t, probe[r], lo, hi), type);
    }
  }
  uint64_t tot;
  (void)block_scan_excl<uint64_t>(c, ws, &tot);
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

// pass 2: the tile re-probes and writes its pairs at tile_off[tile] + (rows before, in
// row order: row r = base + i*THREADS is the i-th row of thread t, rows ordered by (i, t))
__global__ __launch_bounds__(HJ_THREADS) void hj_probe_write_kernel(HjTable t, const int64_t *__restrict__ probe,
                                                                    uint64_t n, int type,
                                                                    const uint64_t *__restrict__ tile_off,
                                                                    int64_t *__restrict__ out_p,
                                                                    int64_t *__restrict__ out_b) {
  __shared__ uint64_t ws[HJ_THREADS / kWave];
  const uint64_t base = (uint64_t)blockIdx.x * HJ_TILE + threadIdx.x;
  uint64_t run = tile_off[blockIdx.x];
  for (int i = 0; i < HJ_ITEMS; ++i) {  // one row per thread per step, rows in order
    const uint64_t r = base + (uint64_t)i * HJ_THREADS;
    uint64_t lo = 0, hi = 0;
    int64_t k = 0;
    uint32_t m = 0, c = 0;
    if (r < n) {
      k = probe[r];
      m = hj_matches(t, k, lo, hi);
      c = hj_out_count(m, type);
    }
    uint64_t tot;
    uint64_t pos = run + block_scan_excl<uint64_t>(c, ws, &tot);
    run += tot;
    if (c) {
      if (type == NUT_JOIN_INNER || (type == NUT_JOIN_LEFT && m)) {
        for (uint64_t j = lo; j < hi; ++j)
          if (t.bkeys[j] == k) {
            out_p[pos] = (int64_t)r;
            out_b[pos] = t.brow[j];
            ++pos;
          }
      } else {
        out_p[pos] = (int64_t)r;
        out_b[pos] = -1;
      }
    }
    __syncthreads();  // ws is reused by the next row's scan
  }
}

__global__ void matched_kernel(const int64_t *__restrict__ bi, uint64_t n, int64_t *__restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = bi[i] >= 0 ? 1 : 0;
}

// 1 where a join pair has a build row, 0 for NULL-extended rows (outer joins; sql_plan.cpp)
nut_status join_matched(nut_ctx *c, const int64_t *bi, uint64_t n, int64_t *out) {
  if (!n) return NUT_OK;
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, c->num_cus * 16ull);
  hipLaunchKernelGGL(matched_kernel, dim3(g), dim3(256), 0, c->stream, bi, n, out);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

__global__ void gather_u64_kernel(const uint64_t *__restrict__ src, const int64_t *__restrict__ idx, uint64_t n,
                                  uint64_t null_bits, uint64_t *__restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t j = idx[i];
    out[i] = j < 0 ? null_bits : src[j];
  }
}

}  // namespace nut

using namespace nut;

struct nut_join {
  nut_ctx *ctx = nullptr;
  void *mem = nullptr;  // table (offsets, bucket keys, row ids) + tile counts / offsets
  HjTable t{};
  const int64_t *probe = nullptr;
  uint64_t np = 0, ntiles = 0, n = 0;
  int type = 0;
  uint64_t *toff = nullptr;
};

namespace {

// exclusive scan of n u32 / u64 values into out[0..n] (out[n] = total)
template <class T>
nut_status excl_scan(nut_ctx *c, const T *in, uint64_t n, uint64_t *out, uint64_t *sums) {
  const uint64_t blocks = (n + SC_TILE - 1) / SC_TILE;
  hipLaunchKernelGGL(scan_reduce_kernel<T>, dim3((unsigned)blocks), dim3(SC_THREADS), 0, c->stream, in, n, sums);
  hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(SC_THREADS), 0, c->stream, sums, blocks);
  hipLaunchKernelGGL(scan_apply_kernel<T>, dim3((unsigned)blocks), dim3(SC_THREADS), 0, c->stream, in, n,
                     (const uint64_t *)sums, out);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

nut_status join_build_count(nut_ctx *c, nut_join *j, const int64_t *build, uint64_t nb) {
  hipStream_t st = c->stream;
  int log2b = 0;  // >= 2 buckets per build row
  while ((1ull << log2b) < 2 * std::max<uint64_t>(nb, 1)) ++log2b;
  const uint64_t nbk = 1ull << log2b;
  const uint64_t ntiles = (j->np + HJ_TILE - 1) / HJ_TILE;
  const uint64_t nsc = std::max<uint64_t>(nbk, ntiles);
  // [counts u32 nbk | offsets u64 nbk+1 | cursors u64 nbk | bkeys nb | brow nb | tile counts u64 |
  //  tile offsets u64 ntiles+1 | scan sums]
  size_t o = 0;
  auto carve = [&](size_t bytes) {
    const size_t r = o;
    o += (bytes + 255) & ~size_t(255);
    return r;
  };
  const size_t o_cnt = carve(nbk * 4), o_off = carve((nbk + 1) * 8), o_cur = carve(nbk * 8), o_bk = carve(nb * 8),
               o_br = carve(nb * 8), o_tc = carve(ntiles * 8), o_to = carve((ntiles + 1) * 8),
               o_sm = carve(((nsc + SC_TILE - 1) / SC_TILE + 1) * 8);
  NUT_HIP(hipMalloc(&j->mem, o));
  char *b = (char *)j->mem;
  uint32_t *cnt = (uint32_t *)(b + o_cnt);
  uint64_t *off = (uint64_t *)(b + o_off), *cur = (uint64_t *)(b + o_cur);
  int64_t *bkeys = (int64_t *)(b + o_bk), *brow = (int64_t *)(b + o_br);
  uint64_t *tcnt = (uint64_t *)(b + o_tc), *sums = (uint64_t *)(b + o_sm);
  j->toff = (uint64_t *)(b + o_to);
  j->ntiles = ntiles;
  NUT_HIP(hipMemsetAsync(cnt, 0, nbk * 4, st));
  const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nb + 255) / 256, c->num_cus * 8ull));
  if (nb) hipLaunchKernelGGL(hj_count_kernel, dim3(g), dim3(256), 0, st, build, nb, log2b, cnt);
  nut_status s = excl_scan<uint32_t>(c, cnt, nbk, off, sums);
  if (s) return s;
  NUT_HIP(hipMemcpyAsync(cur, off, nbk * 8, hipMemcpyDeviceToDevice, st));
  if (nb) hipLaunchKernelGGL(hj_fill_kernel, dim3(g), dim3(256), 0, st, build, nb, log2b, (unsigned long long *)cur,
                             bkeys, brow);
  j->t = HjTable{off, bkeys, brow, log2b};
  j->n = 0;
  if (ntiles) {
    hipLaunchKernelGGL(hj_probe_count_kernel, dim3((unsigned)ntiles), dim3(HJ_THREADS), 0, st, j->t, j->probe, j->np,
                       j->type, tcnt);
    s = excl_scan<uint64_t>(c, tcnt, ntiles, j->toff, sums);
    if (s) return s;
    NUT_HIP(hipMemcpyAsync(c->host_pinned, j->toff + ntiles, 8, hipMemcpyDeviceToHost, st));
    NUT_HIP(hipStreamSynchronize(st));
    j->n = c->host_pinned[0];
  }
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

}  // namespace

extern "C" {

nut_status nut_join_i64(nut_ctx *c, const int64_t *build, uint64_t nb, const int64_t *probe, uint64_t np, int type,
                        nut_join **out, uint64_t *npairs) {
  if (!c || !out || !npairs || (nb && !build) || (np && !probe))
    return fail(NUT_ERR_INVALID_ARG, "nut_join_i64: NULL argument");
  if (type < NUT_JOIN_INNER || type > NUT_JOIN_ANTI) return fail(NUT_ERR_INVALID_ARG, "nut_join_i64: bad join type");
  if (nb >= (1ull << 32)) return fail(NUT_ERR_UNSUPPORTED, "nut_join_i64: build side >= 2^32 rows");
  *out = nullptr;
  DeviceGuard dg(c->device);
  nut_join *j = new nut_join();
  j->ctx = c;
  j->probe = probe;
  j->np = np;
  j->type = type;
  c->timer.begin(c->stream, NUT_KERNEL_JOIN);
  nut_status s = join_build_count(c, j, build, nb);
  c->timer.end(c->stream);
  if (s) {
    nut_join_free(j);
    return s;
  }
  *npairs = j->n;
  *out = j;
  return NUT_OK;
}

nut_status nut_join_write(nut_join *j, int64_t *probe_idx, int64_t *build_idx) {
  if (!j || (j->n && (!probe_idx || !build_idx))) return fail(NUT_ERR_INVALID_ARG, "nut_join_write: NULL argument");
  if (!j->n) return NUT_OK;
  nut_ctx *c = j->ctx;
  DeviceGuard dg(c->device);
  c->timer.begin(c->stream, NUT_KERNEL_JOIN);
  hipLaunchKernelGGL(hj_probe_write_kernel, dim3((unsigned)j->ntiles), dim3(HJ_THREADS), 0, c->stream, j->t, j->probe,
                     j->np, j->type, (const uint64_t *)j->toff, probe_idx, build_idx);
  c->timer.end(c->stream);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

void nut_join_free(nut_join *j) {
  if (!j) return;
  if (j->mem) {
    DeviceGuard dg(j->ctx->device);
    (void)hipStreamSynchronize(j->ctx->stream);
    (void)hipFree(j->mem);
  }
  delete j;
}

nut_status nut_gather_u64(nut_ctx *c, const uint64_t *src, const int64_t *idx, uint64_t n, uint64_t null_bits,
                          uint64_t *out) {
  if (!c || (n && (!idx || !out))) return fail(NUT_ERR_INVALID_ARG, "nut_gather_u64: NULL argument");
  if (n == 0) return NUT_OK;
  DeviceGuard dg(c->device);
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, c->num_cus * 16ull);
  hipLaunchKernelGGL(gather_u64_kernel, dim3(g), dim3(256), 0, c->stream, src, idx, n, null_bits, out);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

}  // extern "C"
