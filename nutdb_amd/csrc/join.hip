// join.hip — hash equi-join on one int64 key.
//
// Build: an open-addressing table of 16-byte slots {key, row} (row = -1: empty), capacity
// the power of two >= 2 x build rows (load <= 0.5), linear probing from the top bits of
// mix64(key).  One agent-scope CAS on the row word claims a slot (memory-side atomic:
// coherent across the XCDs' L2s); the key is stored after the claim and the probe kernel
// runs after the build kernel, so no reader sees a claimed slot without its key.  A probe
// reads one 16-B slot per step: the common case — a unique build key — costs one random
// 128-B line (its run continues in the same line), where a CSR bucket table costs two
// (bucket offsets, then the keys).
//
// The same claim makes duplicate keys separate slots of one run; a check pass (each build
// row walks to its own slot, any equal key before it = duplicates) tells the probe whether
// it may stop at the first match (unique build keys: the PK-FK case) or must walk the run
// to its empty slot.  SEMI / ANTI always stop at the first match.
//
// Probe, when a probe row can match several build rows (repeated build keys under INNER /
// LEFT): ONE pass in probe-row order.  A 512-thread workgroup takes a tile of 4096 probe
// rows by atomic ticket and loads its keys (striped, coalesced).  Runs are walked in
// lock-step rounds: each round issues one slot load for every unfinished row of the lane
// (8 random reads in flight per lane; finished rows issue nothing), then consumes them.
// Each row's output pairs are counted, ranked inside the tile (wave scans + one scan of
// the wave totals) and the tile's global offset comes from decoupled look-back
// (lookback.hpp).  A row with at most one match writes its pair from registers; rows with
// several walk their run again while writing.  Rows come out in probe order with no
// per-row or per-tile count array in HBM.  NUT_OPT_JOIN_PROBE_CFG selects another tile
// shape (tuning).  Otherwise (unique build keys, SEMI / ANTI; NUT_OPT_JOIN_MATCH) in two
// passes: the walks in launch order into a 4-B match array, then the ordered write-out
// from it (hj_match_kernel, below).
//   nut_join_i64 (+ nut_join_write): a count-only pass gives the pair count first, the
//   write pass follows (two probe passes, caller-sized output);
//   nut_join_i64_into: the write pass alone into caller arrays of a given capacity.
//
// Roofline: the probe is bound by random 128-B line fetches (one slot read per probe row
// in the common case, ~1.2 lines with run continuations), not by its sequential bytes —
// see DESIGN.md §4.4 for the measured line rate.
#include <algorithm>
#include <new>
#include <type_traits>

#include "common.hpp"
#include "lookback.hpp"
#include "sort.hpp"

namespace nut {

constexpr uint64_t HJ_EMPTY = ~0ull;

struct HjTable {
  i64x2 *slot;  // .x key, .y build row (-1: empty)
  uint64_t wmask;  // runs wrap inside aligned blocks of wmask + 1 slots (a region, or the table)
  int shift;       // 64 - log2(capacity)
};

// home hash = mix64(key ^ 0x3C6EF372FE94F82A), written as the group-by's owner hash of a
// re-keyed key so the partition kernels (gpart.hpp, kx) compute the same digits; it is
// independent of the multi-GPU owner (owner_hash of the key itself)
constexpr uint64_t HJ_KX = 0x6A09E667F3BCC908ull ^ 0x3C6EF372FE94F82Aull;

__device__ __forceinline__ uint64_t hj_home(int64_t k, const HjTable &t) {
  return owner_hash((uint64_t)k ^ HJ_KX, 0, 1) >> t.shift;
}
__device__ __forceinline__ uint64_t hj_next(uint64_t s, const HjTable &t) {
  return (s & ~t.wmask) | ((s + 1) & t.wmask);
}

// Build and duplicate check: HJ_BITEMS rows per lane in flight (their slot atomics /
// loads are issued together each round, like the probe's run walks).
constexpr int HJ_BITEMS = 4;

// rows: the row id stored per build record (NULL = its index)
__global__ __launch_bounds__(256) void hj_build_kernel(const int64_t *__restrict__ keys, uint64_t n, HjTable t,
                                                       const int64_t *__restrict__ rows) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * HJ_BITEMS) {
    int64_t k[HJ_BITEMS];
    uint64_t s[HJ_BITEMS];
    uint32_t act = 0;
#pragma unroll
    for (int j = 0; j < HJ_BITEMS; ++j) {
      const uint64_t i = i0 + j * stride;
      k[j] = i < n ? __builtin_nontemporal_load(keys + i) : 0;
      s[j] = hj_home(k[j], t);
      act |= (i < n ? 1u : 0u) << j;
    }
    while (act) {  // capacity >= 2n: every row finds an empty slot
      // a plain read of the row words first: occupied slots are skipped without an atomic
      unsigned long long old[HJ_BITEMS];
#pragma unroll
      for (int j = 0; j < HJ_BITEMS; ++j) {
        old[j] = 0;
        if ((act >> j) & 1u) old[j] = reinterpret_cast<const unsigned long long *>(&t.slot[s[j]])[1];
      }
#pragma unroll
      for (int j = 0; j < HJ_BITEMS; ++j)
        if (((act >> j) & 1u) && old[j] == HJ_EMPTY)
          old[j] = atomicCAS(reinterpret_cast<unsigned long long *>(&t.slot[s[j]]) + 1, HJ_EMPTY,
                             (unsigned long long)(rows ? rows[i0 + j * stride] : (int64_t)(i0 + j * stride)));
#pragma unroll
      for (int j = 0; j < HJ_BITEMS; ++j) {
        if (!((act >> j) & 1u)) continue;
        if (old[j] == HJ_EMPTY) {
          reinterpret_cast<int64_t *>(&t.slot[s[j]])[0] = k[j];
          act &= ~(1u << j);
        } else {
          s[j] = hj_next(s[j], t);
        }
      }
    }
  }
}

// Duplicate build keys? Each build row walks its run up to its own slot; a slot with the
// same key before it means the key repeats (of two equal keys, the one placed later in the
// run meets the other).  Unique build keys let the probe stop at its first match.
__global__ __launch_bounds__(256) void hj_dupcheck_kernel(const int64_t *__restrict__ keys, uint64_t n, HjTable t,
                                                          const int64_t *__restrict__ rows,
                                                          uint32_t *__restrict__ dup) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  bool found = false;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * HJ_BITEMS) {
    int64_t k[HJ_BITEMS];
    uint64_t s[HJ_BITEMS];
    uint32_t act = 0;
#pragma unroll
    for (int j = 0; j < HJ_BITEMS; ++j) {
      const uint64_t i = i0 + j * stride;
      k[j] = i < n ? __builtin_nontemporal_load(keys + i) : 0;
      s[j] = hj_home(k[j], t);
      act |= (i < n ? 1u : 0u) << j;
    }
    while (act) {
      i64x2 v[HJ_BITEMS];
#pragma unroll
      for (int j = 0; j < HJ_BITEMS; ++j) {
        v[j] = i64x2{0, -1};
        if ((act >> j) & 1u) v[j] = t.slot[s[j]];
      }
#pragma unroll
      for (int j = 0; j < HJ_BITEMS; ++j) {
        if (!((act >> j) & 1u)) continue;
        const bool mine = v[j].y == (rows ? rows[i0 + j * stride] : (int64_t)(i0 + j * stride));
        found = found || (!mine && v[j].x == k[j]);
        if (mine || v[j].x == k[j]) act &= ~(1u << j);
        s[j] = hj_next(s[j], t);
      }
    }
  }
  if (__any(found) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(dup, 1u);
}

// Region build: the table is cut into regions of HJ_RS slots (128 KB); a region's build
// rows arrive contiguous (hash_partition16 by the home hash's top bits), one workgroup
// builds the region in LDS with LDS atomics — runs wrap inside the region — checks it for
// duplicate keys, and writes it out whole (the table needs no memset).  Persistent (one
// workgroup per CU, nreg / grid regions each): the next region's records are loaded
// before this region's write-out, so their latency hides behind its 128 KB of stores.
constexpr uint32_t HJ_RS = 8192;
constexpr int HJ_RTHREADS = 1024;

// records per lane: the host sends a region at most 7/8 x HJ_RS records
constexpr int HJ_RK = (HJ_RS * 7 / 8 + HJ_RTHREADS - 1) / HJ_RTHREADS;

__global__ __launch_bounds__(HJ_RTHREADS) void hj_region_build_kernel(const int64_t *__restrict__ keys,
                                                                      const int64_t *__restrict__ rows,
                                                                      const uint64_t *__restrict__ region_off,
                                                                      HjTable t, int64_t row_base,
                                                                      uint32_t *__restrict__ dup, uint64_t nreg) {
  __shared__ int64_t s_key[HJ_RS];
  __shared__ unsigned long long s_row[HJ_RS];
  const int tid = threadIdx.x;
  // a region's records, all loads issued together (clamped: no per-record branch) and
  // kept in registers for the duplicate check
  int64_t k[HJ_RK];
  unsigned long long row[HJ_RK];
  auto load = [&](uint64_t r, int64_t (&kk)[HJ_RK], unsigned long long (&rr)[HJ_RK]) {
    const uint64_t lo = region_off[r], hi = region_off[r + 1];
    if (hi <= lo) return;
#pragma unroll
    for (int j = 0; j < HJ_RK; ++j) {
      const uint64_t i = lo + tid + (uint64_t)j * HJ_RTHREADS;
      const uint64_t ic = i < hi ? i : hi - 1;
      kk[j] = keys[ic];
      rr[j] = (unsigned long long)(rows[ic] + row_base);
    }
  };
  uint64_t r = blockIdx.x;
  load(r, k, row);
  for (;;) {
  const uint64_t lo = region_off[r], hi = region_off[r + 1];
  for (uint32_t i = tid; i < HJ_RS; i += HJ_RTHREADS) s_row[i] = HJ_EMPTY;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < HJ_RK; ++j) {
    if (lo + tid + (uint64_t)j * HJ_RTHREADS >= hi) break;
    uint32_t s = (uint32_t)(hj_home(k[j], t) & (HJ_RS - 1));
    for (;;) {  // the host checked that the region has empty slots
      if (s_row[s] == HJ_EMPTY && atomicCAS(&s_row[s], HJ_EMPTY, row[j]) == HJ_EMPTY) {
        s_key[s] = k[j];
        break;
      }
      s = (s + 1) & (HJ_RS - 1);
    }
  }
  __syncthreads();
  bool found = false;
#pragma unroll
  for (int j = 0; j < HJ_RK; ++j) {
    if (lo + tid + (uint64_t)j * HJ_RTHREADS >= hi) break;
    for (uint32_t s = (uint32_t)(hj_home(k[j], t) & (HJ_RS - 1));; s = (s + 1) & (HJ_RS - 1)) {
      if (s_row[s] == row[j]) break;
      if (s_key[s] == k[j]) {
        found = true;
        break;
      }
    }
  }
  if (__any(found) && (tid & (kWave - 1)) == 0) atomicOr(dup, 1u);
  const uint64_t rn = r + gridDim.x;
  if (rn < nreg) load(rn, k, row);  // (the duplicate check above was this region's last use)
  i64x2 *out = t.slot + r * HJ_RS;
  for (uint32_t i = tid; i < HJ_RS; i += HJ_RTHREADS) out[i] = i64x2{s_key[i], (int64_t)s_row[i]};
  if (rn >= nreg) break;
  r = rn;
  __syncthreads();  // every lane's write-out has read s_key / s_row before they are reset
  }
}

// output pairs of one probe row with m matches
__device__ __forceinline__ uint32_t hj_out_count(uint32_t m, int type) {
  switch (type) {
    case NUT_JOIN_INNER: return m;
    case NUT_JOIN_LEFT: return m ? m : 1u;
    case NUT_JOIN_SEMI: return m ? 1u : 0u;
    default: return m ? 0u : 1u;
  }
}

// The ordered probe in two passes (build keys unique, or SEMI / ANTI: at most one build row
// per probe row).  The one-pass ordered kernel below holds each tile's slot of the chip
// from its run walks until its predecessors' totals arrive (look-back), so tiles that
// finished their random reads wait on slower ones: 37 ms vs 29 for the same reads
// unordered.  Here the walks run in launch order with nothing to wait for
// and leave each probe row's build row (-1: none) in `match` (4 B per probe row, coalesced);
// the ordered write-out is then a streaming pass over `match` (hj_probe_kernel<FROM_MATCH>).
template <int HJ_THREADS, int HJ_ITEMS>
__global__ __launch_bounds__(HJ_THREADS, 4) void hj_match_kernel(HjTable t, const int64_t *__restrict__ probe,
                                                                 uint64_t n, uint32_t *__restrict__ match) {
  const uint64_t base = (uint64_t)blockIdx.x * (HJ_THREADS * HJ_ITEMS) + threadIdx.x;
  int64_t key[HJ_ITEMS];
  uint32_t s[HJ_ITEMS], first[HJ_ITEMS];
  uint32_t act = 0;
#pragma unroll
  for (int i = 0; i < HJ_ITEMS; ++i) {
    const uint64_t r = base + (uint64_t)i * HJ_THREADS;
    key[i] = __builtin_nontemporal_load(probe + (r < n ? r : n - 1));
    s[i] = (uint32_t)hj_home(key[i], t);
    first[i] = ~0u;
    act |= (r < n ? 1u : 0u) << i;
  }
  while (__any(act)) {  // (lock-step rounds, as hj_probe_kernel's; every walk stops at its first match)
    i64x2 v[HJ_ITEMS];
#pragma unroll
    for (int i = 0; i < HJ_ITEMS; ++i)
      if ((act >> i) & 1u) v[i] = t.slot[s[i]];
#pragma unroll
    for (int i = 0; i < HJ_ITEMS; ++i) {
      const bool occ = ((act >> i) & 1u) && v[i].y != -1;
      const bool hit = occ && v[i].x == key[i];
      if (hit) first[i] = (uint32_t)v[i].y;
      const bool more = occ && !hit;
      s[i] = more ? (uint32_t)hj_next(s[i], t) : s[i];
      act = more ? act : (act & ~(1u << i));
    }
  }
#pragma unroll
  for (int i = 0; i < HJ_ITEMS; ++i) {
    const uint64_t r = base + (uint64_t)i * HJ_THREADS;
    if (r < n) __builtin_nontemporal_store(first[i], match + r);  // ~0u: no match
  }
}

// WRITE = false: count pass (tile = blockIdx.x, tile totals added to *total).
// WRITE = true: ticket-ordered tiles, look-back offsets, pairs written below `cap`; the
// last tile stores the grand total in *total.
// ANY (with WRITE; NUT_JOIN_ANY_ORDER, aggregates over a join): tiles in launch order, each
// claims its output run with one atomic on *total — no ticket, no look-back chain, no
// status array; pairs come out grouped by tile in completion order.
// FROM_MATCH (with WRITE): no walks — each row's match comes from hj_match_kernel's array.
template <bool WRITE, int HJ_THREADS, int HJ_ITEMS, bool ANY = false, bool FROM_MATCH = false>
__global__ __launch_bounds__(HJ_THREADS, HJ_ITEMS <= 8 ? 4 : 1) void hj_probe_kernel(HjTable t, const int64_t *__restrict__ probe,
                                                              uint64_t n, int type, uint32_t *__restrict__ ticket,
                                                              uint64_t *__restrict__ status, uint32_t ntiles,
                                                              unsigned long long *__restrict__ total,
                                                              int64_t *__restrict__ out_p,
                                                              int64_t *__restrict__ out_b, uint64_t cap,
                                                              uint32_t *__restrict__ err,
                                                              const uint32_t *__restrict__ dup,
                                                              const int64_t *__restrict__ prows,
                                                              const uint32_t *__restrict__ match) {
  static_assert(!FROM_MATCH || (WRITE && !ANY), "the match array feeds the ordered write pass");
  constexpr int HJ_WAVES = HJ_THREADS / kWave;
  constexpr uint32_t HJ_TILE = HJ_THREADS * HJ_ITEMS;
  __shared__ uint64_t s_pre[HJ_ITEMS][HJ_WAVES];
  __shared__ uint64_t s_excl;
  __shared__ uint32_t s_tile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t tile = blockIdx.x;
  if (WRITE && !ANY) {
    if (tid == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    tile = s_tile;
  }
  const uint64_t base = (uint64_t)tile * HJ_TILE + tid;
  int64_t key[HJ_ITEMS];
  uint32_t s[HJ_ITEMS], m[HJ_ITEMS], first[HJ_ITEMS];
  uint32_t act = 0;  // bit i: item i's run not finished
#pragma unroll
  for (int i = 0; i < HJ_ITEMS; ++i) {
    const uint64_t r = base + (uint64_t)i * HJ_THREADS;
    if constexpr (FROM_MATCH) {
      const uint32_t b = __builtin_nontemporal_load(match + (r < n ? r : n - 1));
      key[i] = 0;
      s[i] = 0;
      m[i] = b != ~0u ? 1u : 0u;
      first[i] = b;
      continue;
    }
    // clamped, unconditional: a conditional load compiles to a branch and a wait per item
    key[i] = __builtin_nontemporal_load(probe + (r < n ? r : n - 1));
    s[i] = (uint32_t)hj_home(key[i], t);
    m[i] = 0;
    first[i] = 0;
    act |= (r < n ? 1u : 0u) << i;
  }
  // a probe row stops at its first match when the build keys are unique, and always for
  // SEMI / ANTI (existence is all they need)
  const bool stop_on_hit = type >= NUT_JOIN_SEMI || *dup == 0;
  // walk every item's run in lock-step rounds: each round issues one slot load per item
  // (unconditionally — a finished item re-reads its empty slot from cache — so all of
  // them are in flight together), then consumes them
  while (__any(act)) {
    // finished items issue no request; their v[i] is never read (occ below tests act), so
    // it needs no default — a default merged with the loaded value made the compiler wait
    // for each load before the next (one round trip per item instead of one per round)
    i64x2 v[HJ_ITEMS];
#pragma unroll
    for (int i = 0; i < HJ_ITEMS; ++i)
      if ((act >> i) & 1u) v[i] = t.slot[s[i]];
#pragma unroll
    for (int i = 0; i < HJ_ITEMS; ++i) {
      const bool occ = ((act >> i) & 1u) && v[i].y != -1;
      const bool hit = occ && v[i].x == key[i];
      if (hit) {
        first[i] = m[i] ? first[i] : (uint32_t)v[i].y;
        ++m[i];
      }
      const bool more = occ && !(hit && stop_on_hit);
      s[i] = more ? (uint32_t)hj_next(s[i], t) : s[i];
      act = more ? act : (act & ~(1u << i));
    }
  }
  // ranks inside the tile, rows ordered (item, wave, lane); in-wave exclusive ranks: with the match array every row has at most one pair, so 32
  // bits hold them (and 16 fewer VGPRs at 16 rows per lane)
  using Rank = typename std::conditional<FROM_MATCH, uint32_t, uint64_t>::type;
  Rank ex[HJ_ITEMS];
#pragma unroll
  for (int i = 0; i < HJ_ITEMS; ++i) {
    const Rank c = base + (uint64_t)i * HJ_THREADS < n ? hj_out_count(m[i], type) : 0;
    Rank incl = c;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const Rank y = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += y;
    }
    ex[i] = incl - c;
    if (lane == kWave - 1) s_pre[i][wave] = incl;
  }
  __syncthreads();
  if (wave == 0) {
    // the ITEMS x WAVES wave totals, scanned in (item, wave) order, PER consecutive per lane
    constexpr int E = HJ_ITEMS * HJ_WAVES, PER = E > kWave ? E / kWave : 1;
    static_assert(E <= kWave || PER * kWave == E, "wave totals must fill the lanes");
    uint64_t *flat = &s_pre[0][0];
    uint64_t a[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      a[k] = PER * lane + k < E ? flat[PER * lane + k] : 0;
      sum += a[k];
    }
    uint64_t incl = sum;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const uint64_t y = __shfl_up(incl, off, kWave);
      if (lane >= off) incl += y;
    }
    const uint64_t tot = __shfl(incl, kWave - 1, kWave);
    uint64_t run = incl - sum;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (PER * lane + k < E) flat[PER * lane + k] = run;
      run += a[k];
    }
    if (!WRITE) {
      if (lane == 0 && tot) atomicAdd(total, (unsigned long long)tot);
    } else if (ANY) {
      if (lane == 0) s_excl = tot ? atomicAdd(total, (unsigned long long)tot) : 0;
    } else {
      const uint64_t e = lookback(status, tile, tot, err, lane);
      if (lane == 0) {
        s_excl = e;
        if (tile == ntiles - 1) *total = e + tot;
      }
    }
  }
  if (!WRITE) return;
  __syncthreads();
  const uint64_t off0 = s_excl;
#pragma unroll
  for (int i = 0; i < HJ_ITEMS; ++i) {
    const uint64_t r = base + (uint64_t)i * HJ_THREADS;
    const uint32_t c = r < n ? hj_out_count(m[i], type) : 0;
    if (!c) continue;
    uint64_t pos = off0 + s_pre[i][wave] + ex[i];
    if (pos + c > cap) continue;  // too small: the caller retries with the total
    const int64_t pr = prows ? prows[r] : (int64_t)r;
    if (m[i] == 0 || type >= NUT_JOIN_SEMI) {
      out_p[pos] = pr;
      out_b[pos] = -1;
    } else if (m[i] == 1) {
      out_p[pos] = pr;
      out_b[pos] = (int64_t)first[i];
    } else {
      uint64_t q = hj_home(key[i], t);
      for (i64x2 v = t.slot[q]; v.y != -1; q = hj_next(q, t), v = t.slot[q])
        if (v.x == key[i]) {
          out_p[pos] = pr;
          out_b[pos++] = v.y;
        }
    }
  }
}

// the largest build row id a join carries (brows), as unsigned: the probe keeps a matched
// build row in 32 bits (the match array, the one-pass `first`), so ids must stay < 2^32 - 1
__global__ void max_row_kernel(const int64_t *__restrict__ rows, uint64_t n, unsigned long long *__restrict__ out) {
  uint64_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    m = max(m, (uint64_t)rows[i]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = max(m, (uint64_t)__shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(out, (unsigned long long)m);
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

// out may be idx itself (each lane reads idx[i] before writing out[i]), so neither is
// __restrict__; src must not overlap out
__global__ void gather_u64_kernel(const uint64_t *__restrict__ src, const int64_t *idx, uint64_t n,
                                  uint64_t null_bits, uint64_t *out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t j = idx[i];
    out[i] = j < 0 ? null_bits : src[j];
  }
}

}  // namespace nut

using namespace nut;

namespace {

using HjProbeFn = void (*)(HjTable, const int64_t *, uint64_t, int, uint32_t *, uint64_t *, uint32_t,
                           unsigned long long *, int64_t *, int64_t *, uint64_t, uint32_t *, const uint32_t *,
                           const int64_t *, const uint32_t *);
struct HjCfg {
  int threads;
  uint32_t tile;
  HjProbeFn write, count, any, from_match;
};
template <int T, int I>
constexpr HjCfg hj_make() {
  return HjCfg{T, (uint32_t)(T * I), hj_probe_kernel<true, T, I>, hj_probe_kernel<false, T, I>,
               hj_probe_kernel<true, T, I, true>, hj_probe_kernel<true, T, I, false, true>};
}
// the two-pass ordered probe's walk kernel: threads x rows per lane, the unordered probe's
// shapes (NUT_OPT_JOIN_ANY_CFG picks for both)
struct HjMatchCfg {
  int threads;
  uint32_t tile;
  void (*fn)(HjTable, const int64_t *, uint64_t, uint32_t *);
};
template <int T, int I>
constexpr HjMatchCfg hj_match_make() {
  return HjMatchCfg{T, (uint32_t)(T * I), hj_match_kernel<T, I>};
}
const HjMatchCfg &hj_match_cfg(int i) {
  static const HjMatchCfg cfgs[] = {hj_match_make<256, 4>(), hj_match_make<512, 8>(), hj_match_make<256, 8>(),
                                    hj_match_make<512, 4>(), hj_match_make<128, 4>()};
  return cfgs[i];
}
// its ordered write-out: 512 x 16 tiles (streaming, so the larger tile halves the look-back
// chain; same box, 1e9 probe rows: join 41.04 ms vs 41.99 / 42.47 at 512 x 8,
// profiles/r05/join/cfg_ab.txt).  Its tiles are larger than any ordered shape's, so the
// status array sized at build holds them.
const HjCfg &hj_emit_cfg() {
  static const HjCfg c = hj_make<512, 16>();
  return c;
}
// probe tile shapes (threads x rows per lane); NUT_OPT_JOIN_PROBE_CFG picks one for tuning
// runs.  A join keeps the index it was built with (its status array is sized by the tile).
const HjCfg &hj_cfg(int i) {
  static const HjCfg cfgs[] = {hj_make<512, 8>(), hj_make<256, 8>(), hj_make<256, 16>(), hj_make<512, 16>(),
                               hj_make<256, 4>()};
  return cfgs[i];
}
// the unordered probe's tile shape: no look-back chain to shorten, so the smallest tiles
// with the fewest registers (most waves, most slot loads in flight) — NUT_OPT_JOIN_ANY_CFG
const HjCfg &hj_any_cfg(int i) {
  static const HjCfg cfgs[] = {hj_make<256, 4>(), hj_make<512, 8>(), hj_make<256, 8>(), hj_make<512, 4>(),
                               hj_make<128, 4>()};
  return cfgs[i];
}

}  // namespace

struct nut_join {
  nut_ctx *ctx = nullptr;
  void *mem = nullptr;  // table slots + probe state (status per tile, ticket, error, total)
  size_t mem_bytes = 0;  // (a pooled allocation: pool_take / pool_give)
  HjTable t{};
  const int64_t *probe = nullptr;
  const int64_t *brows = nullptr, *prows = nullptr;  // row ids of the build / probe records (NULL: index)
  uint64_t np = 0, ntiles = 0, n = 0;
  int type = 0;
  bool any_order = false;  // NUT_JOIN_ANY_ORDER: the unordered probe
  bool two_pass = false;   // ordered write in two passes (hj_match_kernel): <= 1 build row per probe row
  int cfg = 0, any_cfg = 0;  // probe tile shapes chosen at build (context options then)
  uint64_t *status = nullptr;
  uint32_t *ticket = nullptr, *err = nullptr, *dup = nullptr;
  unsigned long long *total = nullptr;
  size_t state_bytes = 0;
};

namespace {

nut_status join_build(nut_ctx *c, nut_join *j, const int64_t *build, uint64_t nb) {
  hipStream_t st = c->stream;
  int log2c = 6;  // >= 2 slots per build row, >= 64 slots
  while ((1ull << log2c) < 2 * nb) ++log2c;
  const uint64_t cap = 1ull << log2c;
  j->cfg = (int)c->opt[NUT_OPT_JOIN_PROBE_CFG];
  j->any_cfg = (int)c->opt[NUT_OPT_JOIN_ANY_CFG];
  j->ntiles = (j->np + hj_cfg(j->cfg).tile - 1) / hj_cfg(j->cfg).tile;
  if (j->ntiles > 0xFFFFFFF0ull) return fail(NUT_ERR_UNSUPPORTED, "nut_join_i64: probe side too large");
  // [slots 16 B x cap | dup u32, pad | ticket u32, err u32, total u64 | status u64 x ntiles]
  const size_t o_dup = cap * 16, o_state = o_dup + 16;
  j->state_bytes = 16 + j->ntiles * 8;
  nut_status ps = pool_take(c, o_state + j->state_bytes, &j->mem, &j->mem_bytes);
  if (ps) return ps;
  char *b = (char *)j->mem;
  j->t = HjTable{(i64x2 *)b, cap - 1, 64 - log2c};
  j->ticket = (uint32_t *)(b + o_state);
  j->err = j->ticket + 1;
  j->total = (unsigned long long *)(b + o_state + 8);
  j->status = (uint64_t *)(b + o_state + 16);
  j->dup = (uint32_t *)(b + o_dup);
  NUT_HIP(hipMemsetAsync(j->dup, 0, 16, st));
  // region build for tables of 2^22 .. 2^29 slots (regions of 8192 slots, one 16-bit
  // partition), unless a region would be too full (many equal keys): then global CAS
  const bool region_on = c->opt[NUT_OPT_JOIN_REGION] != 0;
  if (nb && region_on && log2c >= 22 && log2c <= 29) {
    const int rb = log2c - 13;
    const uint64_t nreg = 1ull << rb;
    int64_t *tmp = nullptr;
    NUT_HIP(hipMallocAsync((void **)&tmp, nb * 32, st));
    std::vector<uint64_t> counts;
    nut_status e = hash_partition16(c, build, nb, HJ_KX, tmp, tmp + nb, tmp + 2 * nb, tmp + 3 * nb, counts, j->brows);
    if (e) {
      (void)hipFreeAsync(tmp, st);
      return e;
    }
    std::vector<uint64_t> off(nreg + 1, 0);
    uint64_t mx = 0;
    for (uint64_t r = 0; r < nreg; ++r) {
      uint64_t cnt = 0;
      for (uint64_t q = r << (16 - rb); q < (r + 1) << (16 - rb); ++q) cnt += counts[q];
      off[r + 1] = off[r] + cnt;
      mx = std::max(mx, cnt);
    }
    if (mx <= HJ_RS * 7 / 8) {
      uint64_t *doff = nullptr;
      NUT_HIP(hipMallocAsync((void **)&doff, (nreg + 1) * 8, st));
      NUT_HIP(hipMemcpyAsync(doff, off.data(), (nreg + 1) * 8, hipMemcpyHostToDevice, st));
      j->t.wmask = HJ_RS - 1;
      hipLaunchKernelGGL(hj_region_build_kernel, dim3((unsigned)std::min<uint64_t>(nreg, (uint64_t)c->num_cus)),
                         dim3(HJ_RTHREADS), 0, st, (const int64_t *)(tmp + 2 * nb), (const int64_t *)(tmp + 3 * nb),
                         (const uint64_t *)doff, j->t, (int64_t)0, j->dup, nreg);
      NUT_HIP(hipGetLastError());
      NUT_HIP(hipStreamSynchronize(st));  // `off` is host memory of this frame
      (void)hipFreeAsync(doff, st);
      (void)hipFreeAsync(tmp, st);
      return NUT_OK;
    }
    (void)hipFreeAsync(tmp, st);
  }
  NUT_HIP(hipMemsetAsync(b, 0xFF, cap * 16, st));
  if (nb) {
    const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nb + 255) / 256, c->num_cus * 16ull));
    hipLaunchKernelGGL(hj_build_kernel, dim3(g), dim3(256), 0, st, build, nb, j->t, j->brows);
    if (j->type <= NUT_JOIN_LEFT)
      hipLaunchKernelGGL(hj_dupcheck_kernel, dim3(g), dim3(256), 0, st, build, nb, j->t, j->brows, j->dup);
  }
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

// the two-pass write's match array (4 B per probe row), or NULL when HBM has no room for it
// (the caller then takes the one-pass ordered write, which needs none)
uint32_t *match_buffer(nut_ctx *c, uint64_t np) {
  uint32_t *m = nullptr;
  if (hipMallocAsync((void **)&m, np * 4, c->stream) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return m;
}

// one probe pass; WRITE: pairs below cap into (pi, bi).  Returns the pair count.
nut_status join_probe(nut_join *j, bool write, int64_t *pi, int64_t *bi, uint64_t cap, uint64_t *npairs) {
  nut_ctx *c = j->ctx;
  hipStream_t st = c->stream;
  *npairs = 0;
  if (!j->ntiles) return NUT_OK;
  uint32_t *match = nullptr;
  if (j->any_order && write) {
    NUT_HIP(hipMemsetAsync(j->ticket, 0, 16, st));
    const HjCfg &cf = hj_any_cfg(j->any_cfg);
    const uint64_t nt = (j->np + cf.tile - 1) / cf.tile;
    if (nt > 0x7FFFFFFFull) return fail(NUT_ERR_UNSUPPORTED, "nut_join: probe side too large");
    cf.any<<<dim3((unsigned)nt), dim3(cf.threads), 0, st>>>(j->t, j->probe, j->np, j->type, j->ticket, j->status,
                                                         (uint32_t)nt, j->total, pi, bi, cap, j->err,
                                                         (const uint32_t *)j->dup, j->prows, nullptr);
  } else if (write && j->two_pass && (match = match_buffer(c, j->np)) != nullptr) {
    // two passes (at most one build row per probe row): the walks, then the ordered write-out
    // (no room for the match array: the one-pass form below)
    const HjCfg &cf = hj_emit_cfg();
    const uint64_t nt = (j->np + cf.tile - 1) / cf.tile;
    if (nt > j->ntiles) {
      (void)hipFreeAsync(match, st);
      return fail(NUT_ERR_UNSUPPORTED, "nut_join: write-out tiles exceed the status array");
    }
    const HjMatchCfg &mc = hj_match_cfg(j->any_cfg);
    hipLaunchKernelGGL(mc.fn, dim3((unsigned)((j->np + mc.tile - 1) / mc.tile)), dim3(mc.threads), 0, st, j->t,
                       j->probe, j->np, match);
    NUT_HIP(hipMemsetAsync(j->ticket, 0, 16 + nt * 8, st));
    cf.from_match<<<dim3((unsigned)nt), dim3(cf.threads), 0, st>>>(j->t, j->probe, j->np, j->type, j->ticket,
                                                                 j->status, (uint32_t)nt, j->total, pi, bi, cap,
                                                                 j->err, (const uint32_t *)j->dup, j->prows, match);
    (void)hipFreeAsync(match, st);
  } else {
    NUT_HIP(hipMemsetAsync(j->ticket, 0, j->state_bytes, st));
    const HjCfg &cf = hj_cfg(j->cfg);
    (write ? cf.write : cf.count)<<<dim3((unsigned)j->ntiles), dim3(cf.threads), 0, st>>>(
        j->t, j->probe, j->np, j->type, j->ticket, j->status, (uint32_t)j->ntiles, j->total, pi, bi, cap, j->err,
        (const uint32_t *)j->dup, j->prows, nullptr);
  }
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipMemcpyAsync(c->host_pinned, j->ticket, 16, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  if ((uint32_t)(c->host_pinned[0] >> 32) != 0) return fail(NUT_ERR_TIMEOUT, "nut_join: look-back spin limit hit");
  *npairs = c->host_pinned[1];
  return NUT_OK;
}

nut_status join_begin(nut_ctx *c, const int64_t *build, uint64_t nb, const int64_t *probe, uint64_t np, int type,
                      nut_join **out, const char *who, const int64_t *brows = nullptr,
                      const int64_t *prows = nullptr) {
  const bool any_order = (type & NUT_JOIN_ANY_ORDER) != 0;
  type &= ~NUT_JOIN_ANY_ORDER;
  if (type < NUT_JOIN_INNER || type > NUT_JOIN_ANTI) return fail(NUT_ERR_INVALID_ARG, std::string(who) + ": bad join type");
  if (nb >= (1ull << 31)) return fail(NUT_ERR_UNSUPPORTED, std::string(who) + ": build side >= 2^31 rows");
  nut_join *j = new (std::nothrow) nut_join();
  if (!j) return fail(NUT_ERR_OOM, std::string(who) + ": out of host memory");
  j->ctx = c;
  j->probe = probe;
  j->np = np;
  j->type = type;
  j->any_order = any_order;
  j->brows = brows;
  j->prows = prows;
  nut_status s = NUT_OK;
  if (brows && nb) {  // build row ids must fit the probe's 32-bit match words (fail loudly, never truncate)
    unsigned long long *mx = (unsigned long long *)c->host_pinned + 8;
    unsigned long long *dmx = nullptr;
    hipError_t e = hipMallocAsync((void **)&dmx, 8, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(dmx, 0, 8, c->stream);
    if (e == hipSuccess) {
      const unsigned g = (unsigned)std::min<uint64_t>((nb + 255) / 256, c->num_cus * 8ull);
      hipLaunchKernelGGL(max_row_kernel, dim3(g), dim3(256), 0, c->stream, brows, nb, dmx);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(mx, dmx, 8, hipMemcpyDeviceToHost, c->stream);
    if (dmx) (void)hipFreeAsync(dmx, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) s = hip_fail(e, who);
    else if (*mx >= 0xFFFFFFFFull)
      s = fail(NUT_ERR_UNSUPPORTED, std::string(who) + ": build row ids >= 2^32 - 1 (the probe keeps 32-bit build rows)");
  }
  if (!s) s = join_build(c, j, build, nb);
  // the ordered write in two passes when no probe row can have two build rows
  // (NUT_OPT_JOIN_MATCH; SEMI / ANTI always, INNER / LEFT when the build keys are unique)
  if (!s && !any_order && np && c->opt[NUT_OPT_JOIN_MATCH] != 0) {
    j->two_pass = type >= NUT_JOIN_SEMI;
    if (!j->two_pass) {
      hipError_t e = hipMemcpyAsync(c->host_pinned, j->dup, 4, hipMemcpyDeviceToHost, c->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
      if (e != hipSuccess) s = hip_fail(e, who);
      j->two_pass = s == NUT_OK && *(const uint32_t *)c->host_pinned == 0;
    }
  }
  if (s) {
    nut_join_free(j);
    return s;
  }
  *out = j;
  return NUT_OK;
}

}  // namespace

nut_status nut::join_i64_into_rows(nut_ctx *c, const int64_t *build, const int64_t *brows, uint64_t nb,
                                   const int64_t *probe, const int64_t *prows, uint64_t np, int type,
                                   int64_t *probe_idx, int64_t *build_idx, uint64_t cap, uint64_t *npairs) {
  if (!c || !npairs || (nb && !build) || (np && !probe) || (cap && (!probe_idx || !build_idx)))
    return fail(NUT_ERR_INVALID_ARG, "nut_join_i64_into: NULL argument");
  DeviceGuard dg(c->device);
  nut_join *j = nullptr;
  c->timer.begin(c->stream, NUT_KERNEL_JOIN);
  nut_status s = join_begin(c, build, nb, probe, np, type, &j, "nut_join_i64_into", brows, prows);
  uint64_t n = 0;
  if (!s) s = join_probe(j, true, probe_idx, build_idx, cap, &n);
  c->timer.end(c->stream);
  nut_join_free(j);
  if (s) return s;
  *npairs = n;
  if (n > cap) return fail(NUT_ERR_CAPACITY, "nut_join_i64_into: " + std::to_string(n) + " pairs > capacity " +
                                                std::to_string(cap));
  return NUT_OK;
}

extern "C" {

nut_status nut_join_i64(nut_ctx *c, const int64_t *build, uint64_t nb, const int64_t *probe, uint64_t np, int type,
                        nut_join **out, uint64_t *npairs) {
  if (!c || !out || !npairs || (nb && !build) || (np && !probe))
    return fail(NUT_ERR_INVALID_ARG, "nut_join_i64: NULL argument");
  *out = nullptr;
  DeviceGuard dg(c->device);
  nut_join *j = nullptr;
  c->timer.begin(c->stream, NUT_KERNEL_JOIN);
  nut_status s = join_begin(c, build, nb, probe, np, type, &j, "nut_join_i64");
  if (!s) s = join_probe(j, false, nullptr, nullptr, 0, &j->n);
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
  uint64_t n = 0;
  c->timer.begin(c->stream, NUT_KERNEL_JOIN);
  nut_status s = join_probe(j, true, probe_idx, build_idx, j->n, &n);
  c->timer.end(c->stream);
  if (!s && n != j->n) return fail(NUT_ERR_HIP, "nut_join_write: pair count changed between passes");
  return s;
}

nut_status nut_join_i64_into(nut_ctx *c, const int64_t *build, uint64_t nb, const int64_t *probe, uint64_t np,
                             int type, int64_t *probe_idx, int64_t *build_idx, uint64_t cap, uint64_t *npairs) {
  return join_i64_into_rows(c, build, nullptr, nb, probe, nullptr, np, type, probe_idx, build_idx, cap, npairs);
}

void nut_join_free(nut_join *j) {
  if (!j) return;
  if (j->mem) pool_give(j->ctx, j->mem, j->mem_bytes);
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
