// gpart.hpp — partitioned aggregation for more groups than the on-chip tables hold
// (BASELINE config 3 at G = 1e5 .. 1e7).
//
// The streaming kernel (agg_kernel.hpp) first runs in SPILL mode: it evaluates WHERE and
// the aggregate arguments as always, but appends every passing row to staged arrays
// {k1, [k2], value arrays} instead of hashing it into a table (and counts the first
// partition level's histogram on the way).  The kernels here then
// radix-partition those records by the key hash (one or two 8-bit levels -> 256 or 65536
// partitions of a few hundred groups each), and the streaming kernel runs again in
// SEGMENT mode, one workgroup per partition: every group of a partition lives in that
// workgroup's LDS table, and the block-end merge into the global table inserts each group
// once, with no contention (partitions hold disjoint keys).
#pragma once

#include "common.hpp"
#include "gtable.hpp"

namespace nut {

constexpr int GP_THREADS = 512;
constexpr int GP_ITEMS = 16;
constexpr uint32_t GP_TILE = GP_THREADS * GP_ITEMS;  // 8192 records per scatter tile
constexpr int GP_HTHREADS = 256;
constexpr uint32_t GP_HTILE = 1u << 18;              // records per histogram tile (one flush each)
constexpr int GP_HLOADS = 16;                        // keys in flight per lane in the histogram
constexpr int GP_BINS = 256;
constexpr int GP_MAX_ARR = 3 + NUT_MAX_VALS;         // hash, k1, k2, value arrays

struct GpSeg {  // records [start, start + count) of the current buffer
  uint64_t start, count;
  uint32_t tile0, pad;  // first tile of the segment in the launch's tile table
  // capped layout (no histogram pass): digit d of this segment owns output rows
  // [obase + d * ocap, obase + (d + 1) * ocap)
  uint64_t obase = 0, ocap = 0;
};

struct GpArrays {
  const uint64_t *src[GP_MAX_ARR];  // [0] unused, [1] k1, [2] k2 (two keys), values
  uint64_t *dst[GP_MAX_ARR];
  int narr;
};

// Range digits (the ordered group-by, aggregate.hip groupby_ordered): keys mapped
// monotonically onto 2^14 cells over a sampled range [lo, lo + span] (signed order; keys
// outside are clamped to the end cells, so the order holds and only the balance suffers):
// x = (k ^ 2^63) - lo, clamped to [0, span]; cell = mulhi((x >> t), mul) with mul =
// floor(2^46 / ((span >> t) + 1)).  With the cells split into bits0 + bits1 digits
// (NUT_OPT_GB_L0_BITS, default 7 + 7), level 0's digit is cell >> bits1 and level 1's
// cell & (2^bits1 - 1), so the partitions are in key order.  (The scatter kernel's RANGE
// template flag chooses these digits over the hash's; t is the range shift, 0 included.)
struct GpRange {
  uint64_t lo, span;
  uint32_t mul;
  int t;  // x's shift: (span >> t) < 2^32
  __host__ __device__ __forceinline__ uint32_t cell(uint64_t k) const {
    uint64_t x = (k ^ 0x8000000000000000ull) - lo;
    x = (k ^ 0x8000000000000000ull) < lo ? 0 : (x > span ? span : x);
    return (uint32_t)(((uint64_t)(uint32_t)(x >> t) * mul) >> 32);  // (v_mul_hi_u32)
  }
};

// the partition digit: a byte of the key tuple's owner hash (recomputed, never stored);
// kx (0 for the aggregation) re-keys the hash: the join table's home hash is
// owner_hash(k ^ kx) with its own kx, independent of the multi-GPU owner (kx = 0)
__device__ __forceinline__ uint32_t gp_digit(const uint64_t *k1, const uint64_t *k2, uint64_t i, int shift,
                                             uint64_t kx) {
  return (uint32_t)(owner_hash(k1[i] ^ kx, k2 ? k2[i] : 0, k2 ? 2 : 1) >> shift) & 255u;
}

// 256-bin histogram of (hash >> shift) & 255 per segment (gather: one for all segments)
__global__ __launch_bounds__(GP_HTHREADS) void gp_hist_kernel(const uint64_t *__restrict__ k1,
                                                              const uint64_t *__restrict__ k2,
                                                              const GpSeg *__restrict__ segs,
                                                              const uint32_t *__restrict__ tile_seg, int shift,
                                                              int gather, unsigned long long *__restrict__ hist,
                                                              uint64_t kx) {
  __shared__ uint32_t cnt[GP_BINS];
  const int tid = threadIdx.x;
  cnt[tid] = 0;
  __syncthreads();
  const uint32_t s = tile_seg[blockIdx.x];
  const GpSeg sg = segs[s];
  const uint64_t lo = sg.start + (uint64_t)(blockIdx.x - sg.tile0) * GP_HTILE;
  const uint32_t n = (uint32_t)min<uint64_t>(GP_HTILE, sg.start + sg.count - lo);
  for (uint32_t i = tid; i < n; i += GP_HTHREADS * GP_HLOADS) {
    // unconditional (clamped) non-temporal loads: all GP_HLOADS keys in flight at once
    uint64_t a[GP_HLOADS], b[GP_HLOADS];
#pragma unroll
    for (int j = 0; j < GP_HLOADS; ++j) {
      const uint64_t r = lo + min(i + j * GP_HTHREADS, n - 1);
      a[j] = __builtin_nontemporal_load(k1 + r);
      b[j] = k2 ? __builtin_nontemporal_load(k2 + r) : 0;
    }
#pragma unroll
    for (int j = 0; j < GP_HLOADS; ++j)
      if (i + j * GP_HTHREADS < n)
        atomicAdd(&cnt[(uint32_t)(owner_hash(a[j] ^ kx, b[j], k2 ? 2 : 1) >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (cnt[tid]) atomicAdd(&hist[(gather ? 0 : (uint64_t)s) * GP_BINS + tid], (unsigned long long)cnt[tid]);
}

// Unstable partition of every segment's records by (hash >> shift) & 255: a tile ranks its
// records with LDS atomics and claims each digit's output run with one global atomic on
// the segment's digit cursor; then every array is staged in LDS in digit order (one LDS
// write per record) and written out in coalesced runs.  Persistent (2 workgroups per CU):
// the keys stay in registers from the digit to their own staging, and the next tile's
// keys are fetched while this tile's value arrays go through.
// Gather mode: all segments share one set of 256 cursors (the spilled blocks' regions ->
// one compact partitioned array).
// (VAR: tuning variants for scripts/tune/gp_tune.hip — bit 0 non-temporal stores, bit 1 no
// stores, bit 2 tile-sequential output, bit 3 sequential output after the scattered address
// is computed, bit 5 early loads (one key array: the first value array's loads at the top
// of the tile, in flight while the tile ranks; the next tile's keys right after this
// tile's keys are staged, before their write-out; every write-out a fixed number of
// stores).  The product runs VAR = 1: non-temporal stores measured 7.16-7.24 vs
// 7.34-7.37 ms per 1e9-record level on two boxes, profiles/r03/gp_tune_*.log)
// RANGE: digits (rg.cell(k) >> shift) & (BINS - 1) of one key (GpRange) instead of the hash.
template <int NK, int T, int VAR = 1, int BITS = 8, bool RANGE = false>
__global__ __launch_bounds__(T) void gp_scatter_kernel(GpArrays ar, const GpSeg *__restrict__ segs,
                                                                const uint32_t *__restrict__ tile_seg, uint32_t ntiles,
                                                                int shift, int gather,
                                                                unsigned long long *__restrict__ cursor, uint64_t kx,
                                                                uint64_t ovf, unsigned long long *__restrict__ oflag,
                                                                GpRange rg = GpRange{},
                                                                unsigned long long *__restrict__ acur = nullptr,
                                                                uint64_t acap = 0,
                                                                unsigned long long *__restrict__ acut = nullptr) {
  static_assert(!RANGE || NK == 1, "range digits: one key");
  constexpr uint32_t TILE = T * GP_ITEMS;
  constexpr int BINS = 1 << BITS;  // (the product: GP_BINS = 256)
  static_assert(TILE <= (1u << 24), "slot bits");
  __shared__ uint64_t s_stage[TILE];
  __shared__ uint8_t s_dig[TILE];
  __shared__ uint32_t s_cnt[BINS];
  __shared__ uint32_t s_tex[BINS];
  __shared__ uint64_t s_gb[BINS];
  __shared__ uint32_t s_wsum[BINS / kWave];
  __shared__ uint32_t s_run[(VAR & 16) ? BINS : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if ((VAR & 16) && tid < BINS) s_run[tid] = 0;
  uint64_t k1[GP_ITEMS], k2[NK == 2 ? GP_ITEMS : 1];
  // records of tile tt: [lo, lo + n); item i of this lane is record i * T + tid
  auto tile_range = [&](uint32_t tt, uint64_t &lo, uint32_t &n) {
    const GpSeg g = segs[tile_seg[tt]];
    lo = g.start + (uint64_t)(tt - g.tile0) * TILE;
    n = (uint32_t)min<uint64_t>(TILE, g.start + g.count - lo);
  };
  // unconditional (clamped) loads from one per-tile base: all in flight at once, one
  // 32-bit offset per item
  auto load_arr = [&](const uint64_t *src, uint64_t lo, uint32_t n, uint64_t (&v)[GP_ITEMS]) {
    const uint64_t *b = src + lo;
#pragma unroll
    for (int i = 0; i < GP_ITEMS; ++i) v[i] = __builtin_nontemporal_load(b + min((uint32_t)i * T + tid, n - 1));
  };
  uint32_t t = blockIdx.x;
  if (t >= ntiles) return;
  uint64_t lo;
  uint32_t n;
  tile_range(t, lo, n);
  load_arr(ar.src[1], lo, n, k1);
  if constexpr (NK == 2) load_arr(ar.src[2], lo, n, k2);
  for (;;) {
    // per-item offsets (i * T + tid) are loop-invariant; hoisted out of the tile loop they
    // pinned 16+ registers and pushed the keys into scratch (serialising their loads), so
    // the loop works from an opaque copy of tid
    int tid_ = tid;
    asm volatile("" : "+v"(tid_));
    const int tid = tid_;
    const uint32_t s = tile_seg[t];
    constexpr bool EARLY = (VAR & 32) && NK == 1;
    uint64_t v[GP_ITEMS];
    if constexpr (EARLY)
      if (ar.narr > 3) load_arr(ar.src[3], lo, n, v);  // in flight while the tile ranks
    if (tid < BINS) s_cnt[tid] = 0;
    __syncthreads();
    // rank: sd[i] = digit | in-digit rank << 8, then the tile slot once the digit starts are known
    uint32_t sd[GP_ITEMS];
#pragma unroll
    for (int i = 0; i < GP_ITEMS; ++i) {
      const uint32_t d = RANGE ? (rg.cell(k1[i]) >> shift) & (BINS - 1)
                               : (uint32_t)(owner_hash(k1[i] ^ kx, NK == 2 ? k2[i] : 0, NK) >> shift) & (BINS - 1);
      const uint32_t r = (uint32_t)i * T + tid < n ? atomicAdd(&s_cnt[d], 1u) : 0u;
      sd[i] = d | (r << BITS);
    }
    __syncthreads();
    uint32_t c = 0, incl = 0;
    if (tid < BINS) {
      c = s_cnt[tid];
      incl = c;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
      }
      if (lane == 63) s_wsum[wave] = incl;
    }
    __syncthreads();
    if (tid < BINS) {
      uint32_t add = 0;
#pragma unroll
      for (int w = 0; w < BINS / kWave; ++w) add += (w < wave) ? s_wsum[w] : 0u;
      const uint32_t tex = incl - c + add;
      s_tex[tid] = tex;
      const uint64_t cs = gather ? 0 : (uint64_t)s;
      // (VAR & 16, timing only: per-workgroup sub-regions instead of the global cursor)
      const GpSeg &g0 = segs[s];
      const uint64_t gb = (VAR & 16) ? g0.obase + (uint64_t)tid * g0.ocap + (uint64_t)blockIdx.x * (g0.ocap / gridDim.x) + s_run[tid]
                          : c ? (uint64_t)atomicAdd(&cursor[cs * BINS + tid], (unsigned long long)c) : 0;
      if (VAR & 16) s_run[tid] += c;
      // ovf != 0: the capped layout (no histogram pass; GpSeg obase / ocap).  A run past its
      // digit's rows goes to the scratch rows at ovf (>= one tile of them), and the flag
      // after the cursors tells the host to partition again with a histogram.  With an
      // overflow arena (acur: the ordered group-by) the run is kept instead: it claims rows
      // [ovf + *acur, + c) of the arena (acap rows, scratch after them), which the host
      // aggregates on its own and folds into the result — a heavy key costs its excess
      // rows, not a rerun; only an exhausted arena sets the flag.  The digit's valid rows
      // then end where the first overflowing run would have started (acut[digit] = the
      // least such start: every run claimed after it overflows too), so the rows between
      // there and the region's end, never written, are never read.
      const GpSeg &g = segs[s];
      const bool over = !(VAR & 16) && ovf && c && gb + c > g.obase + (uint64_t)(tid + 1) * g.ocap;
      uint64_t o = gb;
      if (over) {
        const uint64_t ga = acur ? (uint64_t)atomicAdd(acur, (unsigned long long)c) : acap;
        const bool kept = acur && ga + c <= acap;
        if (!kept) atomicOr(oflag, 1ull);
        if (acut) atomicMin(&acut[cs * BINS + tid], (unsigned long long)gb);
        o = ovf + (kept ? ga : acap);
      }
      s_gb[tid] = o - tex;  // out position of tile slot j with digit d = s_gb[d] + j
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < GP_ITEMS; ++i) {
      const uint32_t d = sd[i] & (BINS - 1);
      sd[i] = (sd[i] >> BITS) + s_tex[d];  // the tile slot
      if ((uint32_t)i * T + tid < n) s_dig[sd[i]] = (uint8_t)d;
    }
    // one array through LDS: stage in digit order (its registers are then free), write
    // out coalesced runs.  The first value array loads while the keys are written out,
    // the next tile's keys while the values are.
    auto stage = [&](const uint64_t (&v)[GP_ITEMS]) {
      __syncthreads();  // the previous array's write-out is done with s_stage
#pragma unroll
      for (int i = 0; i < GP_ITEMS; ++i)
        if ((uint32_t)i * T + tid < n) s_stage[sd[i]] = v[i];
      __syncthreads();
    };
    auto flush = [&](uint64_t *dst) {
      // not fully unrolled: the scheduler would hoist every item's LDS reads (and their
      // registers) above the first store
#pragma unroll 2
      for (int i = 0; i < GP_ITEMS; ++i) {
        // (EARLY: unconditional, clamped to the tile's last record — a repeat stores the
        // same word — so that the stores behind a load are a known count)
        const uint32_t j = EARLY ? min((uint32_t)i * T + tid, n - 1) : (uint32_t)i * T + tid;
        if (EARLY || j < n) {
          const uint64_t x = s_stage[j];
          uint64_t o = (VAR & 4) ? lo + j : s_gb[s_dig[j]] + j;
          if (VAR & 8) o = o == ~0ull ? o : lo + j;
          if (VAR & 2) {
            if (x == 0x0123456789ABCDEFull) dst[o] = x;  // (keeps the LDS reads)
          } else if (VAR & 1) {
            __builtin_nontemporal_store(x, &dst[o]);
          } else {
            dst[o] = x;
          }
        }
      }
    };
    stage(k1);
    const uint32_t next = t + gridDim.x;
    uint64_t nlo = 0;
    uint32_t nn = 0;
    if constexpr (EARLY) {  // the key registers are free: the next tile's keys now
      if (next < ntiles) {
        tile_range(next, nlo, nn);
        load_arr(ar.src[1], nlo, nn, k1);
      }
      flush(ar.dst[1]);
    } else {
      if constexpr (NK == 2) {
        flush(ar.dst[1]);
        stage(k2);
      }
      if (ar.narr > 3) load_arr(ar.src[3], lo, n, v);
      flush(ar.dst[NK == 2 ? 2 : 1]);
      if (next < ntiles) {  // the key registers are free
        tile_range(next, nlo, nn);
        load_arr(ar.src[1], nlo, nn, k1);
        if constexpr (NK == 2) load_arr(ar.src[2], nlo, nn, k2);
      }
    }
    for (int a = 3; a < ar.narr; ++a) {
      stage(v);
      if (a + 1 < ar.narr) load_arr(ar.src[a + 1], lo, n, v);
      flush(ar.dst[a]);
    }
    if (next >= ntiles) break;
    __syncthreads();  // s_cnt / s_stage / s_dig / s_gb are reused
    t = next;
    lo = nlo;
    n = nn;
  }
}

// ---------------------------------------------------------------- ordered group-by
// (aggregate.hip groupby_ordered: range-partitioned levels, per-partition ordering, the
// result streamed to the host chunk by chunk)

// m keys at even strides of the column: the sample the range digits are cut from
__global__ void go_sample_kernel(const int64_t *__restrict__ k, uint64_t n, uint32_t m, int64_t *__restrict__ out) {
  const uint64_t step = n / m;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) out[i] = k[i * step];
}

// The heavy-key pass's groups (heavy.hpp) into their partitions' dense regions after the
// chunk's aggregation and before its ordering: hq[j] = heavy key j's partition (global
// index; outside [q0, q0 + nq): another chunk's, or -1: none, the host folds it), appended
// after the partition's own groups (hagg: table-encoded words, as the regions hold them).
// One workgroup, so a region that fills up is cut back after every claim is made: the keys
// that did not fit are flagged in miss[j] (the host folds them).
__global__ __launch_bounds__(1024) void go_heavy_insert_kernel(const int64_t *__restrict__ hk,
                                                               const uint64_t *__restrict__ hagg, uint32_t h, int na,
                                                               const int64_t *__restrict__ hq, uint64_t q0, uint64_t nq,
                                                               unsigned long long *__restrict__ cnt,
                                                               uint64_t *__restrict__ slot, uint64_t *__restrict__ agg,
                                                               uint64_t gstr, uint64_t dregion,
                                                               uint64_t *__restrict__ miss) {
  for (uint32_t j0 = 0; j0 < h; j0 += blockDim.x) {
    const uint32_t j = j0 + threadIdx.x;
    const int64_t q = j < h ? hq[j] : -1;
    const bool mine = q >= (int64_t)q0 && q < (int64_t)(q0 + nq);
    uint64_t idx = 0;
    if (mine) {
      idx = atomicAdd(&cnt[q], 1ull);
      if (idx < dregion) {
        const uint64_t at = (uint64_t)q * dregion + idx;
        slot[at] = (uint64_t)hk[j];
        for (int a = 0; a < na; ++a) agg[(uint64_t)a * gstr + at] = hagg[(uint64_t)j * na + a];
      } else {
        miss[j] = 1;
      }
    }
    __syncthreads();
    if (mine && idx >= dregion) atomicMin(&cnt[q], (unsigned long long)dregion);
    __syncthreads();
  }
}

// Rows per range cell (GpRange: 2^14 cells) of the heavy pass's kept rows: workgroup b
// counts the count[b] rows at row b * chunk of k (heavy.hpp's compacted chunks).  With the
// heavy keys split off, the rest of a skewed distribution still loads its cells unevenly
// (keys of ~1/2 to 2 cell shares), so both levels then lay their regions out from these
// exact counts — no capped regions, no overflow arenas — for 8 B per kept row.
constexpr int GO_HIST_THREADS = 512;
constexpr uint32_t GO_CELLS = 1u << 14;
__global__ __launch_bounds__(GO_HIST_THREADS) void go_cell_hist_kernel(const uint64_t *__restrict__ k,
                                                                       const uint64_t *__restrict__ count,
                                                                       uint64_t chunk, GpRange rg,
                                                                       unsigned long long *__restrict__ cells) {
  __shared__ uint32_t h[GO_CELLS];
  for (uint32_t i = threadIdx.x; i < GO_CELLS; i += GO_HIST_THREADS) h[i] = 0;
  __syncthreads();
  const uint64_t n = count[blockIdx.x];
  const uint64_t *b = k + (uint64_t)blockIdx.x * chunk;
  constexpr int L = 8;
  for (uint64_t i = threadIdx.x; i < n; i += GO_HIST_THREADS * L) {
    uint64_t a[L];  // (clamped loads, all in flight before the first count)
#pragma unroll
    for (int j = 0; j < L; ++j) a[j] = __builtin_nontemporal_load(b + min(i + (uint64_t)j * GO_HIST_THREADS, n - 1));
#pragma unroll
    for (int j = 0; j < L; ++j)
      if (i + (uint64_t)j * GO_HIST_THREADS < n) atomicAdd(&h[rg.cell(a[j])], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < GO_CELLS; i += GO_HIST_THREADS)
    if (h[i]) atomicAdd(&cells[i], (unsigned long long)h[i]);
}

// one workgroup: offs[p] = *run + the groups of the partitions before p, then *run += all
// of them (each thread a run of ceil(np / 1024) consecutive partitions)
__global__ __launch_bounds__(1024) void go_scan_kernel(const unsigned long long *__restrict__ cnt, uint32_t np,
                                                       uint64_t *__restrict__ offs, unsigned long long *__restrict__ run) {
  __shared__ uint64_t ws[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t per = (np + 1023) / 1024, i0 = (uint32_t)tid * per, i1 = min(np, i0 + per);
  uint64_t sum = 0;
  for (uint32_t i = i0; i < i1; ++i) sum += cnt[i];
  uint64_t incl = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) ws[wave] = incl;
  __syncthreads();
  uint64_t add = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    add += w < wave ? ws[w] : 0;
    tot += ws[w];
  }
  const uint64_t base = *run;
  uint64_t e = base + add + incl - sum;
  for (uint32_t i = i0; i < i1; ++i) {
    offs[i] = e;
    e += cnt[i];
  }
  __syncthreads();  // every thread has read *run
  if (tid == 0) *run = base + tot;
}

// one workgroup per partition: its staged groups (unique keys, any order) ordered by key
// and written to the ordered result at offs[p] + rank: keys rk[pos], aggregate words
// ra[pos * na + a] (MIN / MAX of f64 back from their ordered encoding).  A counting sort in
// LDS: each key's bucket is its place in the partition's own [min, max] cut into nb >= n
// buckets (a monotone map, as the sort's MsMap), ranks in the bucket by LDS atomics, a
// scan, then a key's rank = its bucket's start + the keys of its bucket that are smaller
// (~0.6 per bucket: a short loop).  Positions >= cap are not written (the host reports the
// count).  Dynamic LDS: go_order_lds(dregion).
constexpr int GO_ORDER_THREADS = 256;
__host__ __device__ inline uint32_t go_order_nb(uint64_t dregion) {
  uint32_t nb = GO_ORDER_THREADS;
  while (nb < dregion) nb *= 2;
  return nb;
}
inline size_t go_order_lds(uint64_t dregion) { return dregion * 12 + (size_t)go_order_nb(dregion) * 4 + 64; }
__global__ __launch_bounds__(GO_ORDER_THREADS) void go_order_kernel(
    const uint64_t *__restrict__ slot, const uint64_t *__restrict__ agg, uint64_t gstr, uint64_t dregion,
    uint64_t dbase, const unsigned long long *__restrict__ cnt, const uint64_t *__restrict__ offs, int na,
    uint32_t kinds, int64_t *__restrict__ rk, uint64_t *__restrict__ ra, uint64_t cap) {
  extern __shared__ uint64_t s_u[];  // [dregion] keys (sign-flipped), then [nb] bucket counts, [dregion] members
  uint32_t *s_b = (uint32_t *)(s_u + dregion);
  uint32_t *s_m = s_b + go_order_nb(dregion);
  __shared__ uint64_t s_mn[GO_ORDER_THREADS / 64], s_mx[GO_ORDER_THREADS / 64];
  __shared__ uint32_t s_ws[GO_ORDER_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t p = blockIdx.x, n = (uint32_t)cnt[p];
  if (n == 0) return;
  const uint32_t nb = go_order_nb(n);  // buckets: a power of two >= n
  const uint64_t base = (dbase + p) * dregion;
  uint64_t mn = ~0ull, mx = 0;
  for (uint32_t i = tid; i < n; i += GO_ORDER_THREADS) {
    const uint64_t u = slot[base + i] ^ 0x8000000000000000ull;
    s_u[i] = u;
    mn = u < mn ? u : mn;
    mx = u > mx ? u : mx;
  }
  for (uint32_t b = tid; b < nb; b += GO_ORDER_THREADS) s_b[b] = 0;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const uint64_t a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if (lane == 0) {
    s_mn[wave] = mn;
    s_mx[wave] = mx;
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < GO_ORDER_THREADS / 64; ++w) {
    mn = s_mn[w] < mn ? s_mn[w] : mn;
    mx = s_mx[w] > mx ? s_mx[w] : mx;
  }
  const uint64_t span = mx - mn;
  const int sh = span >> 32 ? 64 - __clzll((long long)span) - 32 : 0;
  const uint64_t mulb = ((uint64_t)nb << 32) / ((span >> sh) + 1);  // bucket = ((u - mn) >> sh) * mulb >> 32 < nb
  auto bucket = [&](uint64_t u) { return (uint32_t)((((u - mn) >> sh) * mulb) >> 32); };
  // the keys' ranks in their buckets (kept in registers: <= dregion / 256 keys per thread)
  constexpr int KPT = 17;  // dregion <= 4097 (the host checks)
  uint32_t r[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t i = tid + j * GO_ORDER_THREADS;
    r[j] = i < n ? atomicAdd(&s_b[bucket(s_u[i])], 1u) : 0u;
  }
  __syncthreads();
  // bucket counts -> starts (nb / 256 consecutive buckets per thread)
  const uint32_t per = nb / GO_ORDER_THREADS;
  uint32_t sum = 0;
  for (uint32_t b = 0; b < per; ++b) sum += s_b[tid * per + b];
  uint32_t incl = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) s_ws[wave] = incl;
  __syncthreads();
  uint32_t e = incl - sum;
#pragma unroll
  for (int w = 0; w < GO_ORDER_THREADS / 64; ++w) e += w < wave ? s_ws[w] : 0u;
  for (uint32_t b = 0; b < per; ++b) {
    const uint32_t c = s_b[tid * per + b];
    s_b[tid * per + b] = e;
    e += c;
  }
  __syncthreads();
  // members of every bucket, contiguous from its start
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t i = tid + j * GO_ORDER_THREADS;
    if (i < n) s_m[s_b[bucket(s_u[i])] + r[j]] = i;
  }
  __syncthreads();
  const uint64_t o = offs[p];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint32_t i = tid + j * GO_ORDER_THREADS;
    if (i >= n) continue;
    const uint64_t u = s_u[i];
    const uint32_t b = bucket(u), b0 = s_b[b], b1 = b + 1 < nb ? s_b[b + 1] : n;
    uint32_t rank = b0;
    for (uint32_t q = b0; q < b1; ++q) rank += s_u[s_m[q]] < u;
    const uint64_t pos = o + rank;
    if (pos >= cap) continue;
    rk[pos] = (int64_t)(u ^ 0x8000000000000000ull);
    for (int a = 0; a < na; ++a) {
      uint64_t x = agg[(uint64_t)a * gstr + base + i];
      const int kd = kind_at(kinds, a);
      if (kd == AK_MIN_F64 || kd == AK_MAX_F64) x = ord_to_f64(x);
      ra[pos * na + a] = x;
    }
  }
}

}  // namespace nut
