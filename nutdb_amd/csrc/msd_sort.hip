// msd_sort.hip — SELECT k FROM t ORDER BY k (BASELINE config 5) as a hybrid MSD radix sort:
// a few segmented MSD scatter levels in HBM, then every segment small enough for one
// workgroup is finished on chip.  Replaces the 8-pass LSD sort (sort.hip) as nut_sort_i64.
//
// Why: the LSD sort moves every key through HBM 8 times (16 B/key each)
// and each pass pays a serial decoupled look-back.  For 1.25e9 random keys the hybrid
// moves them twice through HBM plus one on-chip finish:
//     8 (histogram) + 16 (level 0) + 8 (histogram) + 16 (level 1) + 16 (local) = 64 B/key
// instead of 8 + 8 x 16 = 136 B/key.
//
//   * level histograms (ms_hist_kernel): one 512-bin LDS histogram per 256 Ki-key tile of a
//     segment, flushed with global atomics; the first also reduces min / max, so the levels
//     sort (key - base) by its varying bits (a narrow key range is rebased onto 0 and its
//     first digit starts at the top bit of max - min).
//   * plans (ms_plan_kernel): a level's per-segment digit counts become the next level's
//     work lists (scatter again / local-sort size class) on the device.
//   * scatter levels (ms_scatter_kernel): 9-bit digits, 16 Ki-key tiles, persistent; keys
//     only, so a level needs no stability — the local sort re-sorts every segment.  A tile
//     ranks its keys with LDS atomics (one per key), stages them in LDS in digit order and
//     claims each digit's output run with ONE global atomic on the segment's digit cursor:
//     no look-back chain, no spin, progress independent of dispatch order.
//   * local sort (ms_local_kernel, three size classes): a segment's keys in registers are
//     placed at their bucket positions (next varying bits) in LDS, every lane sorts one
//     window of whole buckets with an in-register network (wider windows: half-wave /
//     wave bitonic networks), and the segment is written once, coalesced.  Segments the
//     windows cannot split (heavy duplicates) fall back to ms_lsd_kernel (stable LSD passes
//     in LDS).
// Keys map to u64 with the sign bit flipped (DESC: its complement) on the first load and
// back on the final store.
#include <algorithm>
#include <cstdlib>
#include <utility>
#include <vector>

#include "common.hpp"
#include "sort.hpp"

namespace nut {

constexpr int MH_THREADS = 256;
constexpr uint32_t MH_TILE = 1u << 16;  // keys per copy tile
constexpr uint32_t MH_HTILE = 1u << 18; // keys per histogram tile (one LDS histogram flush each)
constexpr int MH_LOADS = 16;            // keys in flight per lane in the histogram loop
constexpr int MS_THREADS = 1024;
constexpr int MS_ITEMS = 14;
constexpr uint32_t MS_TILE = MS_THREADS * MS_ITEMS;  // keys staged in LDS at a time (14336)
constexpr int MS_BITS = 9;                          // digit width of a scatter level
constexpr int MS_BINS = 1 << MS_BITS;               // 512: MS_TILE / 512 = 28 keys (224 B) per digit per stage
static_assert(MS_BINS <= MS_THREADS, "one scan thread per digit");
// local-sort classes: threads x max items per thread (ms_local_kernel), by segment size.
// The segments of a 1.25e9-key sort (~4768 keys) take class 1: 512 threads x 10 keys, three
// workgroups per CU (51 KB of LDS each: 24 waves, 72 VGPRs), one workgroup per segment —
// scripts/tune/local_tune.hip, 262144 segments of 4768 keys: 4.65-4.67 ms vs 5.13-5.18 for
// round 5's 256 x 20 (12 waves per CU) on the same boxes (profiles/r06/sort/local_tune_*.log;
// round 5: 5.14 vs 6.65 for round 4's persistent 512 x 12 at two per CU)
constexpr int LS_NCLS = 4;
constexpr int LS_S_THREADS = 256, LS_S_ITEMS = 8;     // class 0: <= 2048 keys
constexpr int LS_M_THREADS = 512, LS_M_ITEMS = 10;    // class 1: <= 5120 keys, 3 workgroups per CU
constexpr int LS_M2_THREADS = 512, LS_M2_ITEMS = 12;  // class 2: <= 6144 keys, 2 workgroups per CU
constexpr int LS_L_THREADS = 1024, LS_L_ITEMS = 24;   // class 3: <= 24576 keys
constexpr uint64_t LS_S_CAP = LS_S_THREADS * LS_S_ITEMS;
constexpr uint64_t LS_M_CAP = LS_M_THREADS * LS_M_ITEMS;
constexpr uint64_t LS_M2_CAP = LS_M2_THREADS * LS_M2_ITEMS;
constexpr uint64_t LS_CAP = LS_L_THREADS * LS_L_ITEMS;
// the class of a segment of c keys: 0 .. LS_NCLS - 1, or LS_NCLS when no class holds it
__host__ __device__ constexpr int ls_class(uint64_t c) {
  return c <= LS_S_CAP ? 0 : c <= LS_M_CAP ? 1 : c <= LS_M2_CAP ? 2 : c <= LS_CAP ? 3 : LS_NCLS;
}

// A contiguous run [start, start + count) of one of the buffers.
constexpr uint64_t kSameDst = ~0ull;
struct MsSeg {
  uint64_t start, count;
  uint32_t buf;  // 0: caller's input (raw int64: flip on load), 1: out, 2: tmp, 3: tmp2
  uint32_t aux;  // hist / scatter / copy: first tile of the segment; local sort: hi, the
                 // number of low bits of (key - base) its keys may still differ in
  uint64_t dst = kSameDst;  // local sort / copy: where the sorted run goes in out
                            // (kSameDst: at start — the exact layout)
  uint64_t base = 0;        // local sort: the segment's keys k satisfy 0 <= k - base < 2^aux
};
struct MsBufs {
  const uint64_t *in;
  uint64_t *a;  // out
  uint64_t *b;  // tmp
  uint64_t *c;  // tmp2 (the capped layout's second level)
};
__device__ __forceinline__ uint64_t ms_dst_off(const MsSeg &g) { return g.dst == kSameDst ? g.start : g.dst; }
// The digit of a level: bits [shift, shift + log2(mask + 1)) of (key - base).  Every key
// is >= base (the minimum, or 0), so (key - base) orders like key; subtracting the
// minimum makes the first digit split a narrow key range (a sample-sort rank's) evenly.
struct MsDigit {
  uint64_t base;
  int shift;
  uint32_t mask;
  __device__ __forceinline__ uint32_t operator()(uint64_t k) const { return (uint32_t)((k - base) >> shift) & mask; }
  static constexpr bool kCheck = false;
  static constexpr int kAux = 0;
  __device__ __forceinline__ void setup(uint8_t *) const {}
  __device__ __forceinline__ uint32_t operator()(uint64_t k, const uint8_t *) const { return (*this)(k); }
  uint64_t maxx = ~0ull;
};
// The capped layout's digits: keys known (or sampled) to lie in [base,
// base + span] are mapped monotonically onto 2^18 cells, so that the two capped levels use
// all 512 x 512 regions whatever the span — a sample-sort rank's range, or a column's
// narrow one, as evenly as the full 64-bit range.  x = (k - base) >> t < 2^32 (t = the
// span's bit width - 32, or 0), cell = (x * mul) >> 32 < 2^18 (mul = floor(2^50 / ((span >>
// t) + 1))): one v_mul_hi_u32; level 0's digit = cell >> 9, level 1's = cell & 511.  For the
// full range (base 0, t = 32, mul = 2^18) these are the top two 9-bit digits of k.  Level 0
// flags a key outside the span (k - base > maxx; a key below base wraps above it), whose
// digit is garbage but whose write stays inside its region: the caller sorts again with the
// exact layout.  Cell v holds the keys with (k - base) >> t in [ceil(v 2^32 / mul),
// ceil((v + 1) 2^32 / mul)): ms_plan_capped_kernel gives each cell's segment that base.
// The sample sort's range partition (dist.cpp): bucket = #{splitters <= key} (signed keys,
// flip 0), at most 63 splitters in the kernel arguments (a uniform loop of scalar loads).
// Few buckets would put every key's LDS rank atomic on a handful of counters, so each
// bucket is split into 2^sbits sub-bins by hashed key bits (bin = bucket << sbits | h):
// the bins of one bucket stay adjacent, so a bucket is still one contiguous run.
// The bucket comes from a 4096-entry table over the top 12 bits of the (sign-flipped)
// key, copied to LDS by the kernel (kAux): a cell no splitter falls in holds one bucket;
// a cell with splitters inside (flag 0x80) counts the splitters <= key from its first one.
struct MsSplit {
  int ns, sbits;
  int64_t e[63];
  const uint8_t *tab;  // 4096 cells (device), copied to LDS by setup()
  static constexpr bool kCheck = false;
  static constexpr int kAux = 4096;
  __device__ __forceinline__ void setup(uint8_t *s) const {
    for (int i = threadIdx.x; i < kAux; i += blockDim.x) s[i] = tab[i];
  }
  __device__ __forceinline__ uint32_t operator()(uint64_t k, const uint8_t *lds) const {
    const uint32_t t = lds[(k ^ 0x8000000000000000ull) >> 52];
    uint32_t d = t & 63u;
    if (t & 0x80u)
      while (d < (uint32_t)ns && (int64_t)k >= e[d]) ++d;
    const uint32_t h = (uint32_t)(k ^ (k >> 29) ^ (k >> 43));
    return (d << sbits) | (h & ((1u << sbits) - 1u));
  }
};
struct MsMap {
  uint64_t base;
  uint32_t mul, lim;
  int t, dshift;  // dshift: 9 (level 0) or 0 (level 1)
  uint64_t maxx;  // level 0: ((lim + 1) << t) - 1, the largest k - base in range; level 1: ~0
  static constexpr bool kCheck = true;
  static constexpr int kAux = 0;
  __device__ __forceinline__ void setup(uint8_t *) const {}
  __device__ __forceinline__ uint32_t operator()(uint64_t k) const {
    return (__umulhi((uint32_t)((k - base) >> t), mul) >> dshift) & (MS_BINS - 1);
  }
  __device__ __forceinline__ uint32_t operator()(uint64_t k, const uint8_t *) const { return (*this)(k); }
};

__device__ __forceinline__ const uint64_t *ms_src(const MsBufs &bf, uint32_t buf) {
  return buf == 0 ? bf.in : (buf == 1 ? bf.a : (buf == 2 ? bf.b : bf.c));
}

// ---------------------------------------------------------------- level histogram
template <class DG>
__global__ __launch_bounds__(MH_THREADS) void ms_hist_kernel(MsBufs bf, const MsSeg *__restrict__ segs,
                                                             const uint32_t *__restrict__ tile_seg, DG dg0,
                                                             uint64_t flip, unsigned long long *__restrict__ hist,
                                                             unsigned long long *__restrict__ minmax) {
  __shared__ uint32_t h[MS_BINS];
  __shared__ uint8_t s_aux[DG::kAux > 0 ? DG::kAux : 4];
  const int tid = threadIdx.x;
  dg0.setup(s_aux);
  auto dg = [&](uint64_t k) { return dg0(k, s_aux); };
  for (int i = tid; i < MS_BINS; i += MH_THREADS) h[i] = 0;
  __syncthreads();
  const uint32_t s = tile_seg[blockIdx.x];
  const MsSeg sg = segs[s];
  const uint64_t lo = (uint64_t)(blockIdx.x - sg.aux) * MH_HTILE;
  const uint32_t cnt = (uint32_t)min<uint64_t>(MH_HTILE, sg.count - lo);
  const uint64_t *src = ms_src(bf, sg.buf) + sg.start + lo;
  const uint64_t f = sg.buf == 0 ? flip : 0;
  uint64_t vmin = ~0ull, vmax = 0;
  for (uint32_t i = tid; i < cnt; i += MH_THREADS * MH_LOADS) {
    uint64_t k[MH_LOADS];
#pragma unroll
    for (int j = 0; j < MH_LOADS; ++j)  // unconditional (clamped) loads: a conditional one compiles
      k[j] = __builtin_nontemporal_load(src + min(i + j * MH_THREADS, cnt - 1)) ^ f;  // to a branch + wait per key
#pragma unroll
    for (int j = 0; j < MH_LOADS; ++j) {
      if (i + j * MH_THREADS < cnt) {
        atomicAdd(&h[dg(k[j])], 1u);
        vmin = k[j] < vmin ? k[j] : vmin;
        vmax = k[j] > vmax ? k[j] : vmax;
      }
    }
  }
  if (minmax) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const uint64_t a = __shfl_xor(vmin, off, 64), b = __shfl_xor(vmax, off, 64);
      vmin = a < vmin ? a : vmin;
      vmax = b > vmax ? b : vmax;
    }
    if ((tid & 63) == 0) {
      atomicMin(&minmax[0], (unsigned long long)vmin);
      atomicMax(&minmax[1], (unsigned long long)vmax);
    }
  }
  __syncthreads();
  for (int i = tid; i < MS_BINS; i += MH_THREADS)
    if (h[i]) atomicAdd(&hist[(uint64_t)s * MS_BINS + i], (unsigned long long)h[i]);
}

// ---------------------------------------------------------------- scatter level
// Unstable partition of every listed segment by its digit into the other buffer (in /
// tmp -> out ... see ms_dst; dst_buf >= 0 overrides).  cursor[s][d] starts at the absolute
// position of sub-segment (s, d) and is advanced by one atomic per (tile, digit).
// Capped layout (ocap > 0, no histogram pass): sub-segment (s, d) owns the positions
// [(s * MS_BINS + d) * ocap, + ocap); a run that would pass its end is not written and
// sets *oflag (the host then sorts again with the exact layout).
__device__ __forceinline__ uint64_t *ms_dst(const MsBufs &bf, uint32_t buf, int dst_buf) {
  return dst_buf == 1 ? bf.a : dst_buf == 2 ? bf.b : dst_buf == 3 ? bf.c : (buf == 2 ? bf.a : bf.b);
}
constexpr uint64_t kSkipRun = ~0ull;

// Persistent: workgroup b takes tiles b, b + grid, ...; the next tile's keys are loaded into
// the key registers as soon as the current tile is staged in LDS, so its HBM latency hides
// behind the current tile's write-out (and the segment lookup behind the ranking).
// H = 2: tiles of 2 x MS_TILE keys (2 x MS_ITEMS = 28 keys per lane in registers), staged
// and written out in two halves of the tile's digit order through the same MS_TILE-key LDS
// buffer, so each digit's output run per tile is twice as long (~448 B instead of ~224 B:
// fewer partial 128-B lines).
template <int H, class DG, int T = MS_THREADS>
__global__ __launch_bounds__(T, 2048 / T) void ms_scatter_kernel(MsBufs bf, const MsSeg *__restrict__ segs,
                                                                   const uint32_t *__restrict__ tile_seg, uint32_t ntiles,
                                                                   DG dg0, uint64_t flip,
                                                                   unsigned long long *__restrict__ cursor,
                                                                   int dst_buf = -1, uint64_t ocap = 0,
                                                                   unsigned long long *__restrict__ oflag = nullptr) {
  constexpr int ITEMS = MS_ITEMS * H;
  constexpr uint32_t STAGE = (uint32_t)T * MS_ITEMS;  // keys staged in LDS at a time
  constexpr uint32_t TILE = STAGE * H;
  static_assert(MS_BINS <= T, "one scan thread per digit");
  static_assert(TILE <= 65536, "16-bit ranks");
  __shared__ uint64_t s_keys[STAGE];
  __shared__ uint32_t s_cnt[MS_BINS];
  __shared__ uint32_t s_tex[MS_BINS];
  __shared__ uint64_t s_gb[MS_BINS];
  __shared__ uint32_t s_wsum[MS_BINS / kWave];
  __shared__ uint8_t s_aux[DG::kAux > 0 ? DG::kAux : 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  dg0.setup(s_aux);  // (visible after the loop's first barrier)
  auto dg = [&](uint64_t k) { return dg0(k, s_aux); };
  uint32_t t = blockIdx.x;
  uint64_t key[ITEMS];
  // raw loads: the flip is applied when the tile is ranked, so that a prefetch issued
  // before the current tile's write-out does not wait for its data there
  auto load = [&](uint32_t tt, const MsSeg g) {
    const uint64_t lo = (uint64_t)(tt - g.aux) * TILE;
    const uint32_t cn = (uint32_t)min<uint64_t>(TILE, g.count - lo);
    const uint64_t *sp = ms_src(bf, g.buf) + g.start + lo;
    // an opaque copy of tid: hoisted out of the tile loop, the ITEMS per-item offsets
    // would pin registers the next tile's keys need (spills that wait for the prefetch)
    int tq = tid;
    asm volatile("" : "+v"(tq));
    // every load unconditional (clamped to the tile): all ITEMS stay in flight together
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) key[i] = __builtin_nontemporal_load(sp + min((uint32_t)(i * T + tq), cn - 1));
  };
  uint32_t s = tile_seg[t];
  MsSeg sg = segs[s];
  load(t, sg);
  for (;;) {
    // an opaque copy of tid per tile: tid-derived addresses are recomputed, not pinned in
    // registers (or spilled) across the loop
    int tid_ = tid;
    asm volatile("" : "+v"(tid_));
    const int tid = tid_;
    if (sg.buf == 0 && flip) {  // (uniform)
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) key[i] ^= flip;
    }
    const uint64_t lo = (uint64_t)(t - sg.aux) * TILE;
    const uint32_t cnt = (uint32_t)min<uint64_t>(TILE, sg.count - lo);
    uint64_t *dst = ms_dst(bf, sg.buf, dst_buf);
    const uint32_t next = t + gridDim.x;
    const uint32_t ns = next < ntiles ? tile_seg[next] : 0;
    if (tid < MS_BINS) s_cnt[tid] = 0;
    __syncthreads();
    uint32_t rk[ITEMS / 2];  // ranks in the tile's digit run (< TILE), 16-bit pairs
#pragma unroll
    for (int i = 0; i < ITEMS; i += 2) rk[i / 2] = 0;
    bool bad = false;  // MsMap level 0: a key outside the mapped span
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const uint32_t idx = (uint32_t)i * T + tid;
      if (idx < cnt) {
        rk[i / 2] |= atomicAdd(&s_cnt[dg(key[i])], 1u) << (16 * (i & 1));
        if constexpr (DG::kCheck) bad |= key[i] - dg0.base > dg0.maxx;
      }
      if (i % 8 == 7) __builtin_amdgcn_sched_barrier(0);  // (as in the slot loop below)
    }
    if constexpr (DG::kCheck)
      if (__ballot(bad) && lane == 0) atomicOr(oflag, 1ull);
    __syncthreads();
    uint32_t c = 0, incl = 0;
    if (tid < MS_BINS) {
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
    if (tid < MS_BINS) {
      uint32_t add = 0;
#pragma unroll
      for (int w = 0; w < MS_BINS / kWave; ++w) add += (w < wave) ? s_wsum[w] : 0u;
      const uint32_t tex = incl - c + add;
      s_tex[tid] = tex;
      const uint64_t gb = c ? (uint64_t)atomicAdd(&cursor[(uint64_t)s * MS_BINS + tid], (unsigned long long)c) : 0;
      const bool over = ocap && c && gb + c > ((uint64_t)s * MS_BINS + tid + 1) * ocap;
      if (over) atomicOr(oflag, 1ull);
      s_gb[tid] = over ? kSkipRun : gb - tex;  // out position of tile slot j of this digit = s_gb[d] + j
    }
    __syncthreads();
    // rank -> tile slot, in place (16-bit pairs)
#pragma unroll
    for (int i = 0; i < ITEMS; i += 2) {
      const uint32_t s0 = s_tex[dg(key[i])] + (rk[i / 2] & 0xFFFFu);
      const uint32_t s1 = s_tex[dg(key[i + 1])] + (rk[i / 2] >> 16);
      rk[i / 2] = (s0 & 0xFFFFu) | (s1 << 16);
      // groups of 8: with all ITEMS LDS reads hoisted together their results, the keys
      // and the ranks exceed 128 VGPRs, and the spills wait for the next tile's prefetch
      if (i % 8 == 6) __builtin_amdgcn_sched_barrier(0);
    }
    MsSeg nsg = sg;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      if (h) __syncthreads();  // the previous half's write-out is done with s_keys
#pragma unroll
      for (int i = 0; i < ITEMS; ++i) {
        const uint32_t idx = (uint32_t)i * T + tid;
        const uint32_t slot = (rk[i / 2] >> (16 * (i & 1))) & 0xFFFFu;
        if (idx < cnt && (H == 1 || slot / STAGE == (uint32_t)h)) s_keys[slot % STAGE] = key[i];
      }
      if (h == H - 1 && next < ntiles) {  // the key registers are free: fetch the next tile now
        __builtin_amdgcn_sched_barrier(0);  // (not interleaved with the staging: spills)
        nsg = segs[ns];
        load(next, nsg);
      }
      __syncthreads();
      // H = 2: not fully unrolled, or the scheduler hoists every item's LDS read (and its
      // registers) above the first store while the next tile's 32 keys are in flight
#pragma unroll(H == 1 ? MS_ITEMS : 2)
      for (int i = 0; i < MS_ITEMS; ++i) {
        const uint32_t j = (uint32_t)i * T + tid, jj = j + (uint32_t)h * STAGE;
        if (jj < cnt) {
          const uint64_t k = s_keys[j];
          const uint64_t g = s_gb[dg(k)];
          if (g != kSkipRun) dst[g + jj] = k;  // (non-temporal stores measured 2.4 ms slower per sort)
        }
      }
    }
    if (next >= ntiles) break;
    __syncthreads();  // s_keys / s_gb are reused
    t = next;
    s = ns;
    sg = nsg;
  }
}

// ---------------------------------------------------------------- device-planned level
// After a level's histogram: one block per segment, one thread per digit.  The digit's
// exclusive prefix gives the scatter cursor and the sub-segment it will hold; the
// sub-segment goes straight into the list of its local-sort class (LS_NCLS = too large for one:
// the host takes it to another level).  Replaces a host round trip over every
// (segment, digit) pair — 2^18 of them at the second level of 1.25e9 keys.
__global__ __launch_bounds__(MS_BINS) void ms_plan_kernel(const MsSeg *__restrict__ segs,
                                                          const unsigned long long *__restrict__ hist, int hi,
                                                          uint64_t base,
                                                          unsigned long long *__restrict__ cursor,
                                                          MsSeg *__restrict__ lists, uint64_t cap,
                                                          unsigned int *__restrict__ counts) {
  __shared__ unsigned long long s_wsum[MS_BINS / kWave];
  const int d = threadIdx.x, lane = d & 63, wave = d >> 6;
  const MsSeg sg = segs[blockIdx.x];
  const uint64_t c = hist[(uint64_t)blockIdx.x * MS_BINS + d];
  uint64_t incl = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  uint64_t add = 0;
#pragma unroll
  for (int w = 0; w < MS_BINS / kWave; ++w) add += (w < wave) ? s_wsum[w] : 0ull;
  const uint64_t start = sg.start + incl - c + add;
  cursor[(uint64_t)blockIdx.x * MS_BINS + d] = start;
  // list slots: one atomic per (wave, class present) — a per-thread atomic on four
  // addresses serialised 2^18 claims at the memory side (3 ms)
  const int cls = c == 0 ? -1 : ls_class(c);
#pragma unroll
  for (int k = 0; k <= LS_NCLS; ++k) {
    const uint64_t m = __ballot(cls == k);
    if (!m) continue;
    const int leader = __builtin_ctzll(m);
    unsigned int b = 0;
    if (lane == leader) b = atomicAdd(&counts[k], (unsigned int)__popcll(m));
    b = __shfl(b, leader, 64);
    if (cls == k)
      lists[(uint64_t)k * cap + b + lane_rank(m)] = MsSeg{start, c, sg.buf == 2 ? 1u : 2u, (uint32_t)hi, kSameDst, base};
  }
}

// Capped layout's plan (no histogram pass): after the second capped level, one block per
// first-level segment s, one thread per digit d: the sub-segment's count is its cursor's
// advance over its region start; the exclusive scan over d plus the first-level segment's
// place in out (dbase[s], exact: its count is the first level's cursor advance) gives
// where the sorted run goes.  Lists by local-sort class as ms_plan_kernel; a sub-segment
// too large for every class sets *oflag (the host sorts again with the exact layout).
__global__ __launch_bounds__(MS_BINS) void ms_plan_capped_kernel(const unsigned long long *__restrict__ cursor,
                                                                 const uint64_t *__restrict__ dbase, uint64_t ocap,
                                                                 MsMap m, MsSeg *__restrict__ lists, uint64_t cap,
                                                                 unsigned int *__restrict__ counts,
                                                                 unsigned long long *__restrict__ oflag) {
  __shared__ unsigned long long s_wsum[MS_BINS / kWave];
  const int d = threadIdx.x, lane = d & 63, wave = d >> 6;
  const uint64_t r = (uint64_t)blockIdx.x * MS_BINS + d, start = r * ocap;
  const uint64_t c = cursor[r] - start;
  uint64_t incl = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  uint64_t add = 0;
#pragma unroll
  for (int w = 0; w < MS_BINS / kWave; ++w) add += (w < wave) ? s_wsum[w] : 0ull;
  const uint64_t dst = dbase[blockIdx.x] + incl - c + add;
  const int cls = c == 0 ? -1 : ls_class(c);
  if (cls == LS_NCLS) atomicOr(oflag, 1ull);
  // cell r's keys: (k - m.base) >> m.t in [x0, x1), x_v = ceil(v 2^32 / mul) (the first x with
  // umulhi(x, mul) >= v), x1 capped at lim + 1: the segment's base and the bits that vary
  const uint64_t x0 = ((r << 32) + m.mul - 1) / m.mul;
  const uint64_t x1 = min<uint64_t>((((r + 1) << 32) + m.mul - 1) / m.mul, (uint64_t)m.lim + 1);
  const uint64_t width = x1 > x0 ? (x1 - x0) << m.t : 1;  // < 2^64: at most 2^14 x-steps of 2^t
  const uint64_t sbase = m.base + (x0 << m.t);
  const uint32_t hi = width <= 1 ? 0u : (uint32_t)(64 - __builtin_clzll(width - 1));
#pragma unroll
  for (int k = 0; k < LS_NCLS; ++k) {
    const uint64_t mk = __ballot(cls == k);
    if (!mk) continue;
    const int leader = __builtin_ctzll(mk);
    unsigned int b = 0;
    if (lane == leader) b = atomicAdd(&counts[k], (unsigned int)__popcll(mk));
    b = __shfl(b, leader, 64);
    if (cls == k) lists[(uint64_t)k * cap + b + lane_rank(mk)] = MsSeg{start, c, 3u, hi, dst, sbase};
  }
}

// strided sample of the (flipped) input for the capped layout's admission check
__global__ void ms_sample_kernel(const uint64_t *__restrict__ in, uint64_t n, uint64_t flip, uint32_t m,
                                 uint64_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) out[i] = in[(uint64_t)(((unsigned __int128)i * n) / m)] ^ flip;
}

// ---------------------------------------------------------------- local sort
// One workgroup sorts one segment of <= THREADS * MAXK keys, whose keys agree on every bit
// of (key - base) at or above hi = aux, and writes it to out at the same range.
//
// Main path (MSD split + bitonic windows):
//   1. the keys sit in registers; each takes a rank in its bucket with one LDS atomic, the
//      bucket being the top SB bits of (key - base) below hi (unstable: keys only);
//   2. an exclusive scan gives bucket offsets; buckets are grouped into WINDOWS — the
//      positions from the first bucket start >= q*WS up to the next such start — so a window
//      is a run of whole buckets of about WS + (one bucket) keys;
//   3. the keys are written to LDS (8 B each) at their bucket positions, in at most two
//      rounds of LDS_KEYS keys; every wave then takes windows, loads one into registers
//      (64 or 128 slots, padded with all-ones), sorts it with a bitonic network
//      (full 64-bit compares; xor partners by lane shuffles, partners >= 64 in registers)
//      and stores it straight to out.  Sorting whole buckets in place is sorting the segment,
//      because every key of a bucket is below every key of the next.
// Fallback (a window > 128 keys, or no round split, e.g. heavy duplicates): the segment is
// listed for ms_lsd_kernel — stable LSD passes in LDS (ballot peer ranking, per-wave digit
// counters, exchange by 32-bit halves).
constexpr int LS_WS = 12;           // window stride: windows hold ~WS +- part of a bucket
constexpr int LS_LANE_N = 16;       // windows up to this size are sorted inside one lane
constexpr int LS_MAX_WINDOW = 128;  // largest bitonic network (2 registers per lane)

constexpr int DPP_QUAD_X1 = 0xB1;  // quad_perm [1,0,3,2]: lane ^ 1
constexpr int DPP_QUAD_X2 = 0x4E;  // quad_perm [2,3,0,1]: lane ^ 2
constexpr int DPP_ROR8 = 0x128;    // row_ror:8: lane ^ 8 within 16

// 32-bit DPP move (bound_ctrl: every lane is a valid source for the patterns used here)
template <int CTRL>
__device__ __forceinline__ uint32_t dppm(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
constexpr int DPP_QUAD_M3 = 0x1B;        // quad_perm [3,2,1,0]: lane ^ 3
constexpr int DPP_ROW_HALF_MIRROR = 0x141;  // lane ^ 7 within 8
constexpr int DPP_ROW_MIRROR = 0x140;       // lane ^ 15 within 16
constexpr int DPP_ROW_SHL4 = 0x104, DPP_ROW_SHR4 = 0x114;
// Partner values for the flag-free bitonic network: P = (M, X) selects lane ^ X where the
// first stage of each merge uses the mirror lane ^ (2^m - 1) and the rest lane ^ 2^j.
template <int X>
__device__ __forceinline__ uint32_t lane_x32(uint32_t v) {
  if constexpr (X == 1) return dppm<DPP_QUAD_X1>(v);
  else if constexpr (X == 2) return dppm<DPP_QUAD_X2>(v);
  else if constexpr (X == 3) return dppm<DPP_QUAD_M3>(v);
  else if constexpr (X == 7) return dppm<DPP_ROW_HALF_MIRROR>(v);
  else if constexpr (X == 15) return dppm<DPP_ROW_MIRROR>(v);
  else if constexpr (X == 8) return dppm<DPP_ROR8>(v);
  else if constexpr (X == 4) {
    // banks 0 and 2 of a row (lanes with bit 2 clear) read lane + 4, banks 1 and 3 lane - 4
    const int t = __builtin_amdgcn_update_dpp((int)v, (int)v, DPP_ROW_SHL4, 0xF, 0x5, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(t, (int)v, DPP_ROW_SHR4, 0xF, 0xA, false);
  } else if constexpr (X == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);  // xor 16 in 32
  else if constexpr (X == 31) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x7C1F);    // xor 31 in 32
  else return (uint32_t)__shfl_xor((int)v, X, 64);
}
template <int X>
__device__ __forceinline__ uint64_t lane_x64(uint64_t v) {
  return ((uint64_t)lane_x32<X>((uint32_t)(v >> 32)) << 32) | lane_x32<X>((uint32_t)v);
}
// one compare-exchange stage, partner lane ^ X, lower lane of the pair keeps the minimum
template <int X, int LOWBIT, int NW>
__device__ __forceinline__ void cx64(uint64_t (&v)[NW], int lane) {
  const bool take_min = (lane & LOWBIT) == 0;
#pragma unroll
  for (int r = 0; r < NW; ++r) {
    const uint64_t p = lane_x64<X>(v[r]);
    v[r] = ((v[r] < p) == take_min) ? v[r] : p;
  }
}
// NW independent ascending 64-element sorts (v[r] at lane), flag-free bitonic network:
// merge of block size 2^m = a mirror stage (lane ^ (2^m - 1)) then half-cleaners
// (lane ^ 2^j, j = m-2 .. 0).  The NW networks are interleaved for instruction-level
// parallelism (one alone is a chain of 21 dependent stages).
template <int NW>
__device__ __forceinline__ void wave_bitonic64_multi(uint64_t (&v)[NW], int lane) {
  cx64<1, 1, NW>(v, lane);
  cx64<3, 2, NW>(v, lane);
  cx64<1, 1, NW>(v, lane);
  cx64<7, 4, NW>(v, lane);
  cx64<2, 2, NW>(v, lane);
  cx64<1, 1, NW>(v, lane);
  cx64<15, 8, NW>(v, lane);
  cx64<4, 4, NW>(v, lane);
  cx64<2, 2, NW>(v, lane);
  cx64<1, 1, NW>(v, lane);
  cx64<31, 16, NW>(v, lane);
  cx64<8, 8, NW>(v, lane);
  cx64<4, 4, NW>(v, lane);
  cx64<2, 2, NW>(v, lane);
  cx64<1, 1, NW>(v, lane);
  cx64<63, 32, NW>(v, lane);
  cx64<16, 16, NW>(v, lane);
  cx64<8, 8, NW>(v, lane);
  cx64<4, 4, NW>(v, lane);
  cx64<2, 2, NW>(v, lane);
  cx64<1, 1, NW>(v, lane);
}

// Sort one window of m <= 128 keys in place in LDS with the whole wave: m <= 64 one
// network; otherwise two sorted 64-halves merged by the block-128 mirror stage (lane ^ 63
// across the two registers) and the half-cleaners inside each register.
__device__ __forceinline__ void sort_window(uint64_t *w, uint32_t m, int lane) {
  if (m <= 64) {
    uint64_t v[1] = {(uint32_t)lane < m ? w[lane] : ~0ull};
    wave_bitonic64_multi<1>(v, lane);
    if ((uint32_t)lane < m) w[lane] = v[0];
    return;
  }
  uint64_t v[2] = {w[lane], (uint32_t)(64 + lane) < m ? w[64 + lane] : ~0ull};
  wave_bitonic64_multi<2>(v, lane);
  const uint64_t p = lane_x64<63>(v[1]);
  const uint64_t mn = v[0] < p ? v[0] : p, mx = v[0] < p ? p : v[0];
  v[0] = mn;
  v[1] = lane_x64<63>(mx);
  cx64<32, 32, 2>(v, lane);
  cx64<16, 16, 2>(v, lane);
  cx64<8, 8, 2>(v, lane);
  cx64<4, 4, 2>(v, lane);
  cx64<2, 2, 2>(v, lane);
  cx64<1, 1, 2>(v, lane);
  w[lane] = v[0];
  if ((uint32_t)(64 + lane) < m) w[64 + lane] = v[1];
}

#ifdef NUT_MSD_PROFILE_STOP
__device__ int g_ms_stop;  // msd_tune only: 1 load, 3 + ranks/scans/LDS, 4 + windows, 5 = all but windows
#define MS_STOP(k) (g_ms_stop == (k))
#else
#define MS_STOP(k) false
#endif
#ifdef NUT_MSD_STAMPS  // local_tune only: per-phase shader cycles of the local sort (thread 0 of each workgroup)
__device__ unsigned long long g_ms_stamp[8];
#define MS_STAMP(k)                                        \
  do {                                                     \
    if (tid == 0) {                                        \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();    \
      if ((k) > 0) st_acc[(k) - 1] += t_ - st_last;        \
      st_last = t_;                                        \
    }                                                      \
  } while (0)
#else
#define MS_STAMP(k) \
  do {              \
  } while (0)
#endif

// SB_ / WS_ = 0: the product defaults (bucket bits by capacity, window stride LS_WS)
template <int THREADS, int MAXK, int SB_ = 0, int WS_ = 0, int LK_ = 0>
struct LocalCfg {
  static constexpr int WAVES = THREADS / kWave;
  static constexpr int CAP = THREADS * MAXK;
  static constexpr int LDS_KEYS = LK_ ? LK_ : (CAP < 16384 ? CAP : 16384);  // 8-B keys per round
  // bucket bits (~1-6 keys each) and window stride.  The M class (6144 keys) takes 4096
  // buckets and windows of ~10 keys: scripts/tune/local_tune.hip -DLT_PLAIN on 262144
  // segments of 4768 keys, two runs: 6.53-6.57 ms vs 6.81-6.85 for 2048 buckets / stride 12
  // (profiles/r04/sort/local_tune_plain.log)
  // (<= 5120 keys: 2048 buckets keep the LDS at 51 KB, three workgroups per CU; 512 x 10 at
  // 4096 buckets and two per CU took 6.03 vs 4.66 ms)
  static constexpr int SB = SB_ ? SB_ : (CAP > 5120 ? 12 : CAP > 2048 ? 11 : 9);
  static constexpr int WS = WS_ ? WS_ : (CAP > 4096 && CAP <= 8192 ? 10 : LS_WS);
  static constexpr int NB = 1 << SB;
  static constexpr int BPT = NB / THREADS;  // buckets per thread in the scan
  static_assert(BPT * THREADS == NB && BPT <= 16, "whole buckets per thread");
  static_assert(CAP <= 2 * LDS_KEYS, "at most two rounds");
  static constexpr int WPT = (CAP / WS + THREADS - 1) / THREADS;  // windows per thread
  static_assert(WPT <= 3, "at most three windows per thread");
  // LDS: one round of 8-B keys, bucket counts -> starts, window starts, scan words
  static constexpr int NWIN = CAP / WS + 2;  // window table entries (+ end)
  static constexpr int BYTES = LDS_KEYS * 8 + ((NB + 1) + NWIN + 16 + 2) * 4;
};

// block-wide exclusive scan of one value per thread (THREADS <= 1024); returns the prefix
// and writes the total to *total.  `ws` = 16 words of LDS.
template <int THREADS>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t *ws, uint32_t *total, int tid) {
  const int lane = tid & 63, wave = tid >> 6;
  uint32_t incl = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) ws[wave] = incl;
  __syncthreads();
  uint32_t add = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < THREADS / kWave; ++w) {
    const uint32_t sw = ws[w];
    add += (w < wave) ? sw : 0u;
    tot += sw;
  }
  *total = tot;
  return incl - x + add;
}

// Batcher's odd-even merge sort network on N (power of two) elements, as a compile-time
// list of compare-exchange pairs (N = 32: 191 pairs).
template <int N>
struct OemNet {
  int a[N * N], b[N * N], n = 0;
  constexpr void merge(int lo, int cnt, int r) {
    const int step = r * 2;
    if (step < cnt) {
      merge(lo, cnt, step);
      merge(lo + r, cnt, step);
      for (int i = lo + r; i + r < lo + cnt; i += step) {
        a[n] = i;
        b[n] = i + r;
        ++n;
      }
    } else {
      a[n] = lo;
      b[n] = lo + r;
      ++n;
    }
  }
  constexpr void sort(int lo, int cnt) {
    if (cnt > 1) {
      sort(lo, cnt / 2);
      sort(lo + cnt / 2, cnt / 2);
      merge(lo, cnt, 1);
    }
  }
  constexpr OemNet() : a(), b() { sort(0, N); }
};
template <int N>
struct OemTable {
  static constexpr OemNet<N> net{};
};

// every lane sorts its own N registers ascending: no cross-lane traffic, each compare-
// exchange is v_cmp_lt_u64 + 4 v_cndmask (N = 16: 63 of them).  The pairs are template
// arguments: indexing v[] with values read from the table at run time (a `#pragma unroll`
// loop over net.a[i]) compiled to VGPR-indexed moves — s_set_gpr_idx_on / v_readlane of
// the indices, ~20 instructions per compare-exchange (378 per local-sort kernel in the ISA)
template <int A, int B, int N>
__device__ __forceinline__ void lane_cx(uint64_t (&v)[N]) {
  const uint64_t x = v[A], y = v[B];
  const bool lt = x < y;
  v[A] = lt ? x : y;
  v[B] = lt ? y : x;
}
template <int N, int... I>
__device__ __forceinline__ void lane_sort_net(uint64_t (&v)[N], std::integer_sequence<int, I...>) {
  (lane_cx<OemTable<N>::net.a[I], OemTable<N>::net.b[I], N>(v), ...);
}
template <int N>
__device__ __forceinline__ void lane_sort(uint64_t (&v)[N]) {
  lane_sort_net<N>(v, std::make_integer_sequence<int, OemTable<N>::net.n>{});
}

// Half-wave batches: register r holds window 2r in lanes 0-31 and window 2r+1 in lanes
// 32-63; NR registers = 2*NR windows of <= 32 keys, one 15-stage network each.
template <int NR>
__device__ __forceinline__ void wave_bitonic32_multi(uint64_t (&v)[NR], int lane) {
  cx64<1, 1, NR>(v, lane);
  cx64<3, 2, NR>(v, lane);
  cx64<1, 1, NR>(v, lane);
  cx64<7, 4, NR>(v, lane);
  cx64<2, 2, NR>(v, lane);
  cx64<1, 1, NR>(v, lane);
  cx64<15, 8, NR>(v, lane);
  cx64<4, 4, NR>(v, lane);
  cx64<2, 2, NR>(v, lane);
  cx64<1, 1, NR>(v, lane);
  cx64<31, 16, NR>(v, lane);
  cx64<8, 8, NR>(v, lane);
  cx64<4, 4, NR>(v, lane);
  cx64<2, 2, NR>(v, lane);
  cx64<1, 1, NR>(v, lane);
}

// waves per SIMD the register budget must allow: four, or as many as the workgroups that
// LDS lets share a CU bring (at most eight) for the classes that run more than four
template <int THREADS, int MAXK, int SB_, int WS_, int LK_>
constexpr int ls_min_waves() {
  using C = LocalCfg<THREADS, MAXK, SB_, WS_, LK_>;
  constexpr int w = (163840 / C::BYTES) * C::WAVES / 4;
  return (LK_ || (THREADS == 512 && MAXK <= 10) || (THREADS == 1024 && MAXK <= 5)) && w > 4 ? (w < 8 ? w : 8) : 4;
}
template <int THREADS, int MAXK, bool PREFETCH, int SB_ = 0, int WS_ = 0, int LK_ = 0>
__global__ __launch_bounds__(THREADS, (ls_min_waves<THREADS, MAXK, SB_, WS_, LK_>())) void ms_local_kernel(MsBufs bf, const MsSeg *__restrict__ segs, uint32_t nseg,
                                                           uint64_t flip, uint32_t *__restrict__ fb) {
  using C = LocalCfg<THREADS, MAXK, SB_, WS_, LK_>;
  constexpr int WAVES = C::WAVES, NB = C::NB, SB = C::SB, LS_WS = C::WS;
  __shared__ __attribute__((aligned(16))) char lds[C::BYTES];
  uint64_t *s_keys = (uint64_t *)lds;
  uint32_t *s_off = (uint32_t *)(lds + C::LDS_KEYS * 8);  // [NB + 1] bucket counts -> starts, then c
  uint32_t *s_win = s_off + NB + 1;                        // [NWIN] window starts
  uint32_t *s_ws = s_win + C::NWIN;                        // 16 scan words
  uint32_t *s_misc = s_ws + 16;                            // [0] max window, [1] round split
  // The thread id without a long-lived VGPR: the wave index in an SGPR and the lane from
  // v_mbcnt, recomputed where needed.  Kept in a VGPR across the segment loop, threadIdx.x
  // was spilled and reloaded before the back edge, and that scratch load — issued after
  // the next segment's loads — made the loop head wait for vmcnt(0): for the prefetch
  // and for this segment's write-out stores (in-order counter)
  const int wv_s = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  auto cur_tid = [&]() -> int {  // (volatile: recomputed where used, never hoisted and spilled)
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return (wv_s << 6) | l;
  };
  const int tid = cur_tid(), lane = tid & 63, wave = wv_s;
  uint64_t key[MAXK];
#ifdef NUT_MSD_STAMPS
  uint64_t st_last = 0, st_acc[7] = {0, 0, 0, 0, 0, 0, 0};
#endif
  // segment g's keys into registers: item i of lane l in wave w = position w*64*K + i*64 + l.
  // Raw loads only: the flip and the padding of positions past the count are applied when
  // the segment is processed (finish_load), so a prefetch does not wait for its data here
  auto load = [&](const MsSeg g) {
    int tq = cur_tid();  // opaque: the item offsets are recomputed, not kept (or spilled) in registers
    asm volatile("" : "+v"(tq));
    const uint32_t cc = (uint32_t)g.count, kk = (cc + THREADS - 1) / THREADS;
    const uint32_t pp = (uint32_t)(tq >> 6) * kWave * kk + (tq & 63);
    const uint64_t *sp = ms_src(bf, g.buf) + g.start;
    // unconditional (clamped) loads, so that all MAXK are in flight at once
#pragma unroll
    for (int i = 0; i < MAXK; ++i) key[i] = __builtin_nontemporal_load(sp + min(pp + (uint32_t)i * kWave, cc - 1));
  };
  auto finish_load = [&](const MsSeg g, const int ftid) {
    const uint32_t cc = (uint32_t)g.count, kk = (cc + THREADS - 1) / THREADS;
    const uint32_t pp = (uint32_t)wv_s * kWave * kk + (uint32_t)(ftid & 63);
    const uint64_t ff = g.buf == 0 ? flip : 0;
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      const uint32_t p = pp + (uint32_t)i * kWave;
      key[i] = ((uint32_t)i < kk && p < cc) ? (key[i] ^ ff) : ~0ull;
    }
  };
  // One step of the persistent loop: sort segment sg (when `active`), and fetch the next
  // segment's keys (PREFETCH, has_next) as soon as this one's are staged in LDS, so their
  // latency hides behind the window sorts and the write-out.  Every path — a segment of
  // equal keys, one for ms_lsd_kernel, the loop's first step that only fetches — passes
  // the ONE load site below, and the write-out issues a fixed number of stores: the
  // compiler then knows how many memory operations follow the loads, so the next step
  // waits for its keys but not for this step's stores (vmcnt counts both, in order).
  // Every condition is block-uniform.
  auto process = [&](const bool active, const uint32_t sidx, const MsSeg sg, const MsSeg nsg, const bool has_next) {
  // an opaque copy of tid per segment: tid-derived addresses kept across the loop were
  // spilled, and a spill reloaded after the prefetch waited for the prefetch (vmcnt is in
  // order), which made it synchronous
  int tq = cur_tid();
  asm volatile("" : "+v"(tq));
  const int tid = tq, lane = tid & 63, wave = wv_s;
  bool work = active;
  MS_STAMP(0);
  const uint32_t c = (uint32_t)sg.count;
  const uint32_t K = (c + THREADS - 1) / THREADS;
  const uint32_t pw = (uint32_t)wave * kWave * K + lane;
  uint64_t *dst = bf.a + ms_dst_off(sg);
  const int hi = (int)sg.aux;   // the keys agree on every bit of (key - base) at or above hi
  const uint64_t base = sg.base;
  auto bucket = [&](uint64_t k) -> uint32_t { return (uint32_t)(((k - base) << (64 - hi)) >> (64 - SB)); };
  uint32_t rk[(MAXK + 1) / 2];  // ranks in the bucket, 16-bit pairs
  uint32_t nq = 0, split = 0, mid = 0;
  if (work) {
    finish_load(sg, tid);
    if (hi == 0) {  // every key equal: copy
#pragma unroll
      for (int i = 0; i < MAXK; ++i) {
        const uint32_t p = pw + (uint32_t)i * kWave;
        if ((uint32_t)i < K && p < c) dst[p] = key[i] ^ flip;
      }
      work = false;
    }
  }
  if (work && MS_STOP(1)) {
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < MAXK; ++i)
      if ((uint32_t)i < K) x ^= key[i];
    dst[tid] = x;
    work = false;
  }
  if (work) {
    // ---- 1. bucket ranks: the top SB of the hi bits of (key - base) that may differ
    //         (fewer than SB: zero-padded, so only some buckets are used)
#pragma unroll
    for (int j = 0; j < C::BPT; ++j) s_off[C::BPT * tid + j] = 0;
    if (tid == 0) {
      s_misc[0] = 0;
      s_misc[1] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MAXK; i += 2) rk[i / 2] = 0;
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      const uint32_t p = pw + (uint32_t)i * kWave;
      if ((uint32_t)i < K && p < c) rk[i / 2] |= atomicAdd(&s_off[bucket(key[i])], 1u) << (16 * (i & 1));
    }
    __syncthreads();
    MS_STAMP(1);
    // ---- 2. bucket starts (BPT consecutive buckets per thread) and windows
    {
      uint32_t cb[C::BPT], sum = 0;
#pragma unroll
      for (int j = 0; j < C::BPT; ++j) {
        cb[j] = s_off[C::BPT * tid + j];
        sum += cb[j];
      }
      uint32_t tot;
      uint32_t e = block_excl_scan<THREADS>(sum, s_ws, &tot, tid);
      __syncthreads();  // every count read before the starts overwrite them
      // Window q starts at the first bucket start >= q * WS: the bucket b whose end
      // (start + count) is the first >= q * WS > its start owns every q with q * WS in
      // (start_b, end_b], and window q then starts at end_b (the next bucket's start).  Each
      // thread assigns the windows its own buckets end — no search; usually none or one.
      const uint32_t nqq = (c + LS_WS - 1) / LS_WS;
#pragma unroll
      for (int j = 0; j < C::BPT; ++j) {
        s_off[C::BPT * tid + j] = e;
        const uint32_t end = e + cb[j];
        for (uint32_t q = e / LS_WS + 1; q * LS_WS <= end && q < nqq; ++q) s_win[q] = end;
        e = end;
      }
      if (tid == 0) {
        s_off[NB] = c;
        s_win[0] = 0;
        s_win[nqq] = c;
      }
    }
    __syncthreads();
    nq = (c + LS_WS - 1) / LS_WS;
    {  // the largest window and the last window that starts inside the first round: a wave
       // maximum, then one LDS atomic per wave (512 atomics on one word serialised)
      uint32_t mw = 0, ms = 0;
#pragma unroll
      for (int j = 0; j < C::WPT; ++j) {
        const uint32_t q = (uint32_t)tid + (uint32_t)j * THREADS;
        if (q < nq) {
          const uint32_t wa = s_win[q], wb = s_win[q + 1];
          mw = max(mw, wb - wa);
          if (wa <= (uint32_t)C::LDS_KEYS) ms = max(ms, q);
        }
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        mw = max(mw, (uint32_t)__shfl_xor((int)mw, off, 64));
        ms = max(ms, (uint32_t)__shfl_xor((int)ms, off, 64));
      }
      if (lane == 0) {
        atomicMax(&s_misc[0], mw);
        atomicMax(&s_misc[1], ms);
      }
    }
    __syncthreads();
    MS_STAMP(2);
    // rounds: windows [0, split) then [split, nq) with at most LDS_KEYS keys each
    split = c > (uint32_t)C::LDS_KEYS ? s_misc[1] : nq;
    mid = split < nq ? s_win[split] : c;
    if (s_misc[0] > (uint32_t)LS_MAX_WINDOW || c - mid > (uint32_t)C::LDS_KEYS) {
      if (tid == 0) fb[1 + atomicAdd(&fb[0], 1u)] = sidx;  // to ms_lsd_kernel
      work = false;
    }
  }
  if (work) {
    // ---- 3. keys to their bucket positions: round 0's into LDS, round 1's parked in out at
    //         their final range (L2-resident; safe in place, every key is in registers)
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      const uint32_t p = pw + (uint32_t)i * kWave;
      if ((uint32_t)i < K && p < c) {
        const uint32_t pos = s_off[bucket(key[i])] + ((rk[i / 2] >> (16 * (i & 1))) & 0xFFFFu);
        if (pos < mid)
          s_keys[pos] = key[i];
        else
          dst[pos] = key[i];
      }
    }
  }
  // the key registers are free: the one load site, unconditional (the last step reloads
  // its own segment) — under a branch, the registers' merge with the unloaded path
  // compiled to copies that waited for the loads right here
  if (PREFETCH) load(nsg);
  MS_STAMP(3);
  if (work && MS_STOP(3)) {
    __syncthreads();
    dst[tid] = s_keys[tid];
    work = false;
  }
  if (!work) return;
  for (int round = 0; round < 2; ++round) {
    const uint32_t rbase = round ? mid : 0;
    const uint32_t w0 = round ? split : 0, w1 = round ? nq : split;
    if (w0 >= w1) break;
    if (round) {  // round 0's windows are done with LDS: bring the parked keys back
      __syncthreads();
      for (uint32_t j = tid; j < c - mid; j += THREADS) s_keys[j] = ld_agent(dst + mid + j);  // L1-bypassing
    }
    __syncthreads();
    // one window per thread (nq <= THREADS): each lane sorts its window of <= 32 keys in
    // its own registers, the rare larger window goes through a wave-wide network; sorted
    // windows go back to LDS, then the round is copied out coalesced
#pragma unroll 1
    for (int j = 0; j < C::WPT && !MS_STOP(5); ++j) {
      const uint32_t t = w0 + (uint32_t)tid + (uint32_t)j * THREADS;
      const uint32_t wa = t < w1 ? s_win[t] - rbase : 0, wm = t < w1 ? s_win[t + 1] - s_win[t] : 0;
      const bool mine = wm > 1 && wm <= (uint32_t)LS_LANE_N;
      if (__ballot(mine)) {
        uint64_t v[LS_LANE_N];
#pragma unroll
        for (int i = 0; i < LS_LANE_N; ++i) v[i] = (mine && (uint32_t)i < wm) ? s_keys[wa + i] : ~0ull;
        lane_sort<LS_LANE_N>(v);
#pragma unroll
        for (int i = 0; i < LS_LANE_N; ++i)
          if (mine && (uint32_t)i < wm) s_keys[wa + i] = v[i];
      }
      // windows of LANE_N+1 .. 32 keys: eight at a time, two per register (half-waves)
      for (uint64_t mid32 = __ballot(wm > (uint32_t)LS_LANE_N && wm <= 32); mid32;) {
        // register r: window 2r in lanes 0-31, window 2r+1 in lanes 32-63; the window's
        // start / length are wave-uniform (readlane into SGPRs), one VGPR pair per register
        uint32_t mg[4], ag[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          uint32_t m2[2], a2[2];
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int l = mid32 ? __builtin_ctzll(mid32) : 0;
            m2[hh] = mid32 ? (uint32_t)__builtin_amdgcn_readlane((int)wm, l) : 0u;
            a2[hh] = mid32 ? (uint32_t)__builtin_amdgcn_readlane((int)wa, l) : 0u;
            mid32 &= mid32 - 1;
          }
          mg[r] = lane < 32 ? m2[0] : m2[1];
          ag[r] = lane < 32 ? a2[0] : a2[1];
        }
        const uint32_t h = (uint32_t)lane & 31;
        uint64_t v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = h < mg[r] ? s_keys[ag[r] + h] : ~0ull;
        wave_bitonic32_multi<4>(v, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (h < mg[r]) s_keys[ag[r] + h] = v[r];
      }
      for (uint64_t big = __ballot(wm > 32); big; big &= big - 1) {  // rare: one by one
        const int l = __builtin_ctzll(big);
        sort_window(s_keys + __shfl(wa, l, 64), __shfl(wm, l, 64), lane);
      }
    }
    __syncthreads();
    MS_STAMP(4);
    if (MS_STOP(4)) continue;
    const uint32_t rend = round ? c : mid;
#ifndef NUT_MSD_DYNAMIC_WRITEOUT  // (scripts/tune/local_tune.hip A/B: the round-4 loop)
    if constexpr (PREFETCH && C::LDS_KEYS == C::CAP) {
#else
    if constexpr (false) {
#endif
      // one round of <= CAP keys: exactly MAXK stores per lane, clamped to the last key
      // (repeats store the same value): a store loop of data-dependent length would leave
      // the compiler no count of the operations behind the next segment's loads
      const uint32_t last = rend - rbase - 1;
      const int tw = cur_tid();
#pragma unroll
      for (int i = 0; i < MAXK; ++i) {
        const uint32_t j = min((uint32_t)(i * THREADS + tw), last);
        __builtin_nontemporal_store(s_keys[j] ^ flip, &dst[rbase + j]);
      }
    } else {
      for (uint32_t j = tid; j < rend - rbase; j += THREADS) __builtin_nontemporal_store(s_keys[j] ^ flip, &dst[rbase + j]);
    }
  }
  MS_STAMP(5);
  };
  if constexpr (!PREFETCH) {  // one segment per workgroup (grid = nseg)
    if (blockIdx.x >= nseg) return;
    const MsSeg sg = segs[blockIdx.x];
    load(sg);
    process(true, blockIdx.x, sg, sg, false);
    return;
  }
  // persistent: segments blockIdx.x, + gridDim.x, ...; the first step only fetches
  uint32_t nidx = blockIdx.x;
  if (nidx >= nseg) return;
  MsSeg sg{}, nsg = segs[nidx];
  uint32_t sidx = 0;
  bool active = false;
  for (;;) {
    const bool has_next = nidx < nseg;
    process(active, sidx, sg, has_next ? nsg : sg, has_next);
    if (!has_next) break;
    __syncthreads();  // LDS is reused by the next segment
    MS_STAMP(6);
    sidx = nidx;
    sg = nsg;
    active = true;
    nidx += gridDim.x;
    if (nidx < nseg) nsg = segs[nidx];
  }
#ifdef NUT_MSD_STAMPS
  if (tid == 0)
    for (int k = 0; k < 7; ++k) atomicAdd(&g_ms_stamp[k], (unsigned long long)st_acc[k]);
#endif
}

// Fallback local sort: the segments ms_local_kernel listed in fb[1 ..] (fb[0] = count)
// get stable LSD passes in LDS.  Item i of lane l in wave w sits at canonical position
// w*64*K + i*64 + l; positions >= count hold all-ones padding, which a stable sort keeps
// behind every real key.
constexpr int LSD_BINS = 256;  // 8-bit passes

template <int THREADS, int MAXK>
__global__ __launch_bounds__(THREADS) void ms_lsd_kernel(MsBufs bf, const MsSeg *__restrict__ segs, uint64_t flip,
                                                         const uint32_t *__restrict__ fb) {
  using C = LocalCfg<THREADS, MAXK>;
  constexpr int WAVES = C::WAVES;
  __shared__ uint32_t s_x[C::CAP];
  __shared__ uint32_t s_wcnt[WAVES][LSD_BINS];
  __shared__ uint32_t s_tex[LSD_BINS];
  __shared__ uint32_t s_wsum[LSD_BINS / kWave];
  __shared__ uint64_t s_wmm[WAVES][2];
  // persistent over the listed segments (grid = min(count, a few per CU)): most launches
  // find none, and a grid of one workgroup per possible segment cost ~0.1 ms per sort
  for (uint32_t blk = blockIdx.x; blk < fb[0]; blk += gridDim.x) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const MsSeg sg = segs[fb[1 + blk]];
    const uint32_t c = (uint32_t)sg.count;
    const uint32_t K = (c + THREADS - 1) / THREADS;
    const uint32_t pw = (uint32_t)wave * kWave * K + lane;
    const uint64_t *src = ms_src(bf, sg.buf) + sg.start;
    uint64_t *dst = bf.a + ms_dst_off(sg);
    const uint64_t f = sg.buf == 0 ? flip : 0;
    uint32_t lo[MAXK], hi[MAXK], pos[MAXK];
    uint64_t mn = ~0ull, mx = 0;
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      const uint32_t p = pw + (uint32_t)i * kWave;
      const uint64_t v = src[min(p, c - 1)] ^ f;  // unconditional: the loads overlap
      if ((uint32_t)i < K && p < c) {
        mn = v < mn ? v : mn;
        mx = v > mx ? v : mx;
      }
      lo[i] = (uint32_t)v;
      hi[i] = (uint32_t)(v >> 32);
    }
    // the segment's key range: passes over bits [0, nbits) of x = key - min; padding
    // (positions >= count) is x = all ones, behind every real key in every pass
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const uint64_t a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
    }
    if (lane == 0) {
      s_wmm[wave][0] = mn;
      s_wmm[wave][1] = mx;
    }
    __syncthreads();
    uint64_t kmin = s_wmm[0][0], kmax = s_wmm[0][1];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) {
      kmin = s_wmm[w][0] < kmin ? s_wmm[w][0] : kmin;
      kmax = s_wmm[w][1] > kmax ? s_wmm[w][1] : kmax;
    }
    const int nbits = kmax == kmin ? 0 : 64 - __builtin_clzll(kmax - kmin);
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      const uint32_t p = pw + (uint32_t)i * kWave;
      const uint64_t x = ((uint32_t)i < K && p < c) ? ((((uint64_t)hi[i] << 32) | lo[i]) - kmin) : ~0ull;
      lo[i] = (uint32_t)x;
      hi[i] = (uint32_t)(x >> 32);
    }
    auto digit = [&](int i, int shift) -> uint32_t {
      return (uint32_t)((((uint64_t)hi[i] << 32) | lo[i]) >> shift) & 255u;
    };
    for (int shift = 0; shift < nbits; shift += 8) {
      for (int i = tid; i < WAVES * LSD_BINS; i += THREADS) (&s_wcnt[0][0])[i] = 0;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < MAXK; ++i) {
        if ((uint32_t)i < K) {
          const uint32_t d = digit(i, shift);
          uint64_t peers = ~0ull;
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            const uint64_t bb = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? bb : ~bb;
          }
          const uint32_t before = lane_rank(peers);
          const uint32_t prior = s_wcnt[wave][d];  // all peers read before the leader writes
          pos[i] = prior + before;
          if (before == 0) s_wcnt[wave][d] = prior + (uint32_t)__popcll(peers);
        }
      }
      __syncthreads();
      uint32_t tot = 0, incl = 0;
      if (tid < LSD_BINS) {
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
          const uint32_t x = s_wcnt[w][tid];
          s_wcnt[w][tid] = tot;  // exclusive prefix over waves
          tot += x;
        }
        incl = tot;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const uint32_t y = __shfl_up(incl, off, 64);
          if (lane >= off) incl += y;
        }
        if (lane == 63) s_wsum[wave] = incl;
      }
      __syncthreads();
      if (tid < LSD_BINS) {
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < LSD_BINS / kWave; ++w) add += (w < wave) ? s_wsum[w] : 0u;
        s_tex[tid] = incl - tot + add;
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < MAXK; ++i) {
        if ((uint32_t)i < K) {
          const uint32_t d = digit(i, shift);
          pos[i] += s_tex[d] + s_wcnt[wave][d];
          s_x[pos[i]] = lo[i];
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < MAXK; ++i)
        if ((uint32_t)i < K) lo[i] = s_x[pw + (uint32_t)i * kWave];
      __syncthreads();
#pragma unroll
      for (int i = 0; i < MAXK; ++i)
        if ((uint32_t)i < K) s_x[pos[i]] = hi[i];
      __syncthreads();
#pragma unroll
      for (int i = 0; i < MAXK; ++i)
        if ((uint32_t)i < K) hi[i] = s_x[pw + (uint32_t)i * kWave];
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      const uint32_t p = pw + (uint32_t)i * kWave;
      if ((uint32_t)i < K && p < c) dst[p] = ((((uint64_t)hi[i] << 32) | lo[i]) + kmin) ^ flip;
    }
    __syncthreads();  // LDS is reused by the next segment
  }
}

// Segments whose keys are all equal (every varying digit consumed): out = key ^ flip.
__global__ __launch_bounds__(MH_THREADS) void ms_copy_kernel(MsBufs bf, const MsSeg *__restrict__ segs,
                                                             const uint32_t *__restrict__ tile_seg, uint64_t flip) {
  const MsSeg sg = segs[tile_seg[blockIdx.x]];
  const uint64_t lo = (uint64_t)(blockIdx.x - sg.aux) * MH_TILE;
  const uint32_t cnt = (uint32_t)min<uint64_t>(MH_TILE, sg.count - lo);
  const uint64_t *src = ms_src(bf, sg.buf) + sg.start + lo;
  uint64_t *dst = bf.a + ms_dst_off(sg) + lo;
  const uint64_t f = sg.buf == 0 ? 0 : flip;  // the caller's input is not flipped
  for (uint32_t i = threadIdx.x; i < cnt; i += MH_THREADS) dst[i] = src[i] ^ f;
}

// ---------------------------------------------------------------- host side
#ifndef NUT_MSD_KERNELS_ONLY  // scripts/tune/msd_tune.hip includes the kernels alone
namespace {

// Per-phase device tables in ctx->sort_meta.  Every phase's uploads and launches are
// stream-ordered after the previous phase's kernels, so each phase reuses the region from
// offset 0; growing it synchronises first (the old allocation may still be in use).
struct MetaArena {
  nut_ctx *c;
  size_t off = 0;
  std::vector<std::vector<char>> keep;  // host copies live until the sort returns

  static size_t align(size_t x) { return (x + 255) & ~size_t(255); }
  // A phase reuses the region from offset 0 while the previous phase's kernels may still
  // read their tables from it (the exact layout's first scatter runs while the next level
  // is planned): wait for them first.  The uploads are stream-ordered anyway, but
  // hipMemcpyAsync from pageable memory makes no such promise for every size.
  nut_status begin(size_t total) {
    off = 0;
    NUT_HIP(hipStreamSynchronize(c->stream));
    if (total > c->sort_meta.bytes) {
      nut_status s = c->sort_meta.reserve(total);
      if (s) return s;
    }
    return NUT_OK;
  }
  void *alloc(size_t bytes) {
    void *p = (char *)c->sort_meta.ptr + off;
    off += align(bytes);
    return p;
  }
  template <class T>
  nut_status upload(const std::vector<T> &v, T **dev) {
    if (off + align(v.size() * sizeof(T)) > c->sort_meta.bytes)  // begin() was sized too small
      return fail(NUT_ERR_UNSUPPORTED, "nut_sort_i64: device table arena overflow");
    *dev = (T *)alloc(v.size() * sizeof(T));
    if (v.empty()) return NUT_OK;
    keep.emplace_back((const char *)v.data(), (const char *)(v.data() + v.size()));
    NUT_HIP(hipMemcpyAsync(*dev, keep.back().data(), v.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return NUT_OK;
  }
};

// tile table: tile -> segment; sets seg.aux = first tile
uint64_t tile_table(std::vector<MsSeg> &segs, uint32_t tile, std::vector<uint32_t> &tiles) {
  tiles.clear();
  for (uint32_t s = 0; s < segs.size(); ++s) {
    segs[s].aux = (uint32_t)tiles.size();
    const uint64_t nt = (segs[s].count + tile - 1) / tile;
    tiles.insert(tiles.end(), nt, s);
  }
  return tiles.size();
}

}  // namespace

// Local sorts: PF = persistent (as many workgroups as fit on the device, each walking the
// list with stride gridDim.x, the next segment's keys prefetched), else one workgroup per
// segment.
template <int T, int K, bool PF>
static void launch_class(nut_ctx *c, const MsBufs &bf, const MsSeg *d, unsigned n, uint64_t flip, uint32_t *fb) {
  static int per_cu = 0;        // resident workgroups per CU (occupancy query, once)
  if (per_cu == 0) {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, ms_local_kernel<T, K, PF>, T, 0) != hipSuccess || b < 1) b = 1;
    per_cu = b;
  }
  const unsigned grid = PF ? (unsigned)std::min<uint64_t>(n, (uint64_t)c->num_cus * per_cu) : n;
  hipLaunchKernelGGL((ms_local_kernel<T, K, PF>), dim3(grid), dim3(T), 0, c->stream, bf, d, n, flip, fb);
  hipLaunchKernelGGL((ms_lsd_kernel<T, K>), dim3((unsigned)std::min<uint64_t>(n, (uint64_t)c->num_cus * 2)), dim3(T), 0,
                     c->stream, bf, d, flip, (const uint32_t *)fb);
}

// local sorts of n segments listed in device memory (a device-planned level's class list)
// (only the S class is persistent: for the M classes one workgroup per segment measured
// 5.14 vs 5.73 ms (256x20) and 6.21-6.29 vs 6.56-6.65 ms (512x12) over 262144 segments of
// 4768 keys, profiles/r05/sort/local_tune_sweep.log — the prefetch's extra registers and its
// loop-carried loads cost more than the launch slots they save; the L class has no
// registers to spare for a second key set)
static nut_status launch_local_dev(nut_ctx *c, const MsBufs &bf, uint64_t flip, const MsSeg *d, unsigned n,
                                   uint32_t *fb, int cls) {
  if (n == 0) return NUT_OK;
  NUT_HIP(hipMemsetAsync(fb, 0, 4, c->stream));
  if (cls == 0)
    launch_class<LS_S_THREADS, LS_S_ITEMS, true>(c, bf, d, n, flip, fb);
  else if (cls == 1)
    launch_class<LS_M_THREADS, LS_M_ITEMS, false>(c, bf, d, n, flip, fb);
  else if (cls == 2)
    launch_class<LS_M2_THREADS, LS_M2_ITEMS, false>(c, bf, d, n, flip, fb);
  else
    launch_class<LS_L_THREADS, LS_L_ITEMS, false>(c, bf, d, n, flip, fb);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

static nut_status launch_local(nut_ctx *c, MetaArena &ar, const MsBufs &bf, uint64_t flip,
                               const std::vector<MsSeg> &segs, int cls) {
  if (segs.empty()) return NUT_OK;
  MsSeg *d;
  nut_status s = ar.upload(segs, &d);
  if (s) return s;
  uint32_t *fb = (uint32_t *)ar.alloc((segs.size() + 1) * 4);
  NUT_HIP(hipMemsetAsync(fb, 0, 4, c->stream));
  return launch_local_dev(c, bf, flip, d, (unsigned)segs.size(), fb, cls);
}


// Scatter tiles are staged and written in two halves (ms_scatter_kernel<2>): ~512-B digit
// runs instead of 256 (29.24 -> 28.72 ms per 1.25e9-key sort, round-2 same-box A/B)
static constexpr int ms_halves() { return 2; }

static void launch_scatter(hipStream_t st, unsigned grid, const MsBufs &bf, const MsSeg *segs, const uint32_t *tiles,
                           uint32_t ntiles, const MsDigit &dg, uint64_t flip, unsigned long long *cur) {
  hipLaunchKernelGGL((ms_scatter_kernel<ms_halves(), MsDigit>), dim3(grid), dim3(MS_THREADS), 0, st, bf, segs, tiles, ntiles, dg,
                     flip, cur);
}

// One device-planned level over `big` (segments whose sizes the host knows): histogram,
// plan (cursors + class lists on the device), scatter, local sorts of the listed classes.
// Only the four class counts come back to the host (read while the scatter runs); the
// sub-segments too large for a local sort are returned in `over` for another level.
static nut_status device_level(nut_ctx *c, MetaArena &ar, const MsBufs &bf, const MsDigit &dg, uint64_t flip,
                               std::vector<MsSeg> &big, std::vector<MsSeg> &over) {
  hipStream_t st = c->stream;
  over.clear();
  std::vector<uint32_t> tiles;
  const uint64_t nht = tile_table(big, MH_HTILE, tiles);
  std::vector<uint32_t> stiles;
  std::vector<MsSeg> sbig = big;
  const uint64_t nst = tile_table(sbig, MS_TILE * ms_halves(), stiles);
  if (nht > 0x7FFFFFFFull || nst > 0x7FFFFFFFull) return fail(NUT_ERR_UNSUPPORTED, "nut_sort_i64: too many tiles");
  const uint64_t ns = big.size(), cap = ns * MS_BINS;
  const size_t hbytes = ns * MS_BINS * 8;
  nut_status s = ar.begin(2 * MetaArena::align(ns * sizeof(MsSeg)) + MetaArena::align(tiles.size() * 4) +
                          MetaArena::align(stiles.size() * 4) + 2 * MetaArena::align(hbytes) +
                          MetaArena::align((LS_NCLS + 1) * cap * sizeof(MsSeg)) +
                          LS_NCLS * MetaArena::align((cap + 1) * 4) + 1024);
  if (s) return s;
  MsSeg *dseg, *dsseg;
  uint32_t *dtile, *dstile;
  if ((s = ar.upload(big, &dseg)) || (s = ar.upload(tiles, &dtile)) || (s = ar.upload(sbig, &dsseg)) ||
      (s = ar.upload(stiles, &dstile)))
    return s;
  unsigned long long *dhist = (unsigned long long *)ar.alloc(hbytes);
  unsigned long long *dcur = (unsigned long long *)ar.alloc(hbytes);
  MsSeg *lists = (MsSeg *)ar.alloc((LS_NCLS + 1) * cap * sizeof(MsSeg));
  unsigned int *counts = (unsigned int *)ar.alloc(4 * (LS_NCLS + 1));
  uint32_t *fb[LS_NCLS];
  for (auto &f : fb) f = (uint32_t *)ar.alloc((cap + 1) * 4);
  NUT_HIP(hipMemsetAsync(dhist, 0, hbytes, st));
  NUT_HIP(hipMemsetAsync(counts, 0, 4 * (LS_NCLS + 1), st));
  uint64_t total = 0;
  for (const MsSeg &sg : big) total += sg.count;
  hipLaunchKernelGGL(ms_hist_kernel<MsDigit>, dim3((unsigned)nht), dim3(MH_THREADS), 0, st, bf, (const MsSeg *)dseg,
                     (const uint32_t *)dtile, dg, flip, dhist, (unsigned long long *)nullptr);
  hipLaunchKernelGGL(ms_plan_kernel, dim3((unsigned)ns), dim3(MS_BINS), 0, st, (const MsSeg *)dseg,
                     (const unsigned long long *)dhist, dg.shift, dg.base, dcur, lists, cap, counts);
  NUT_HIP(hipGetLastError());
  hipEvent_t ev = nullptr;
  NUT_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  uint32_t *hc = (uint32_t *)c->host_pinned;
  hipError_t e = hipMemcpyAsync(hc, counts, 4 * (LS_NCLS + 1), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipEventRecord(ev, st);
  if (e == hipSuccess)
    launch_scatter(st, (unsigned)std::min<uint64_t>(nst, (uint64_t)c->num_cus), bf, (const MsSeg *)dsseg,
                   (const uint32_t *)dstile, (uint32_t)nst, dg, flip, dcur);
  if (e == hipSuccess) e = hipGetLastError();
  if (e == hipSuccess) e = hipEventSynchronize(ev);  // the counts, while the scatter runs
  (void)hipEventDestroy(ev);
  if (e != hipSuccess) return hip_fail(e, "nut_sort_i64 (device-planned level)");
  uint32_t cnt[LS_NCLS + 1];
  for (int k = 0; k <= LS_NCLS; ++k) cnt[k] = hc[k];
  c->sort_bytes += 8 * total + 16 * total;
  ++c->sort_levels;
  for (int cls = LS_NCLS - 1; cls >= 0; --cls)
    if ((s = launch_local_dev(c, bf, flip, lists + (uint64_t)cls * cap, cnt[cls], fb[cls], cls))) return s;
  if (cnt[LS_NCLS]) {  // sub-segments too large for a local sort: to the host, for another level
    over.resize(cnt[LS_NCLS]);
    NUT_HIP(hipMemcpyAsync(over.data(), lists + (uint64_t)LS_NCLS * cap, cnt[LS_NCLS] * sizeof(MsSeg),
                           hipMemcpyDeviceToHost, st));
    NUT_HIP(hipStreamSynchronize(st));
  }
  uint64_t over_keys = 0;
  for (const MsSeg &sg : over) over_keys += sg.count;
  c->sort_bytes += 16 * (total - over_keys);
  return NUT_OK;
}

constexpr uint64_t kCappedMin = 1ull << 25;  // smaller inputs: the exact layout (its passes are short)

// a capped scatter level at T threads per workgroup (NUT_OPT_SORT_BD: 512 = two per CU)
template <class DG, int T>
static void capped_scatter_t(hipStream_t st, unsigned grid, const MsBufs &bf, const MsSeg *segs, const uint32_t *tiles,
                             uint32_t nt, const DG &dg, uint64_t flip, unsigned long long *cur, int dst_buf,
                             uint64_t ocap, unsigned long long *oflag) {
  hipLaunchKernelGGL((ms_scatter_kernel<ms_halves(), DG, T>), dim3(grid), dim3(T), 0, st, bf, segs, tiles, nt, dg, flip,
                     cur, dst_buf, ocap, oflag);
}
template <class DG>
static void capped_scatter(nut_ctx *c, uint64_t nt, const MsBufs &bf, const MsSeg *segs, const uint32_t *tiles,
                           const DG &dg, uint64_t flip, unsigned long long *cur, int dst_buf, uint64_t ocap,
                           unsigned long long *oflag) {
  const bool half = c->opt[NUT_OPT_SORT_BD] == 512;
  const unsigned grid = (unsigned)std::min<uint64_t>(nt, (uint64_t)c->num_cus * (half ? 2 : 1));
  if (half)
    capped_scatter_t<DG, 512>(c->stream, grid, bf, segs, tiles, (uint32_t)nt, dg, flip, cur, dst_buf, ocap, oflag);
  else
    capped_scatter_t<DG, MS_THREADS>(c->stream, grid, bf, segs, tiles, (uint32_t)nt, dg, flip, cur, dst_buf, ocap, oflag);
}

// The capped layout's key map (MsMap) for keys in [lo, hi] of the flipped key space; false
// when the span is too narrow for 2^18 cells (the exact layout then runs).
static bool capped_map(uint64_t lo, uint64_t hi, MsMap &m) {  // (m.dshift = 9: level 0)
  if (hi < lo || hi - lo < (1ull << 18)) return false;
  const uint64_t span = hi - lo;
  const int bw = 64 - __builtin_clzll(span);
  const int t = bw > 32 ? bw - 32 : 0;
  const uint64_t lim = span >> t;  // < 2^32
  const uint64_t mul = (1ull << 50) / (lim + 1);  // (2^18, 2^32): lim >= 2^18
  m = MsMap{lo, (uint32_t)mul, (uint32_t)lim, t, 9, ((lim + 1) << t) - 1};  // (2^64 wraps to ~0)
  return true;
}
// host copy of MsMap's cell (level-0 digit * 512 + level-1 digit)
static uint32_t capped_cell(const MsMap &m, uint64_t k) {
  return (uint32_t)(((uint64_t)(uint32_t)((k - m.base) >> m.t) * m.mul) >> 32);
}

// Capped two-level layout: large inputs whose keys spread evenly over their
// range (in a strided sample) skip both histogram passes.  The keys' range is the sample's
// [min, max] widened by 1/1024 of its span on each side, intersected with the caller's
// bounds when it knows them (a sample-sort rank's splitters); MsMap spreads it over 2^18
// cells.  Level 0 scatters `in` by the cell's top 9 bits into 512 regions of ocap0 rows of
// tmp (about 1.1 x an even share each); level 1 scatters every region by the low 9 bits
// into 512 regions of ocap1 rows of tmp2; the local sorts read those regions and write each
// sorted run to its exact place in out, found by a scan of the level-1 cursors
// (ms_plan_capped_kernel).  48 B/key instead of 64.  A key outside the range, a region
// overflow (a key distribution the sample did not show), a sub-segment too large for a
// local sort or scratch that does not fit returns NUT_ERR_CAPACITY without a message: the
// caller sorts again with the exact layout (`in` is never written).
static nut_status msd_sort_capped(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n, uint64_t flip,
                                  const uint64_t *bounds) {
  hipStream_t st = c->stream;
  constexpr uint32_t kSample = 16384;
  MetaArena ar{c};
  nut_status s = ar.begin(MetaArena::align(kSample * 8) + 1024);
  if (s) return s;
  uint64_t *dsamp = (uint64_t *)ar.alloc(kSample * 8);
  hipLaunchKernelGGL(ms_sample_kernel, dim3(kSample / 256), dim3(256), 0, st, (const uint64_t *)in, n, flip, kSample,
                     dsamp);
  NUT_HIP(hipGetLastError());
  std::vector<uint64_t> samp(kSample);
  NUT_HIP(hipMemcpyAsync(samp.data(), dsamp, kSample * 8, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  MsMap m0;
  {  // the key range, then admission: no digit value holds more than twice its share
    uint64_t smin = ~0ull, smax = 0;
    for (uint64_t k : samp) {
      smin = std::min(smin, k);
      smax = std::max(smax, k);
    }
    const uint64_t d = (smax - smin) >> 10;
    uint64_t lo = smin >= d ? smin - d : 0, hi = smax <= ~0ull - d ? smax + d : ~0ull;
    if (bounds) {
      lo = std::max(lo, bounds[0]);
      hi = std::min(hi, bounds[1]);
    }
    if (!capped_map(lo, hi, m0)) return NUT_ERR_CAPACITY;
    std::vector<uint32_t> h0(MS_BINS, 0), h1(MS_BINS, 0);
    for (uint64_t k : samp) {
      if (k < lo || k > hi) return NUT_ERR_CAPACITY;  // outside the caller's bounds: not a capped input
      const uint32_t cell = capped_cell(m0, k);
      ++h0[cell >> MS_BITS];
      ++h1[cell & (MS_BINS - 1)];
    }
    const uint32_t lim = 2 * kSample / MS_BINS;
    for (int d = 0; d < MS_BINS; ++d)
      if (h0[d] > lim || h1[d] > lim) return NUT_ERR_CAPACITY;
  }
  // scratch that does not fit is a reason for the exact layout (1.25 x n), not a failure
  auto reserve = [&](Scratch &sc, size_t bytes) -> nut_status {
    if (sc.reserve(bytes, false) == NUT_OK) return NUT_OK;
    (void)hipGetLastError();
    c->sort_tmp2.release();
    return NUT_ERR_CAPACITY;
  };
  // ---- level 0: in -> tmp, 512 capped regions
  const uint64_t ocap0 = ((n / MS_BINS) * 11 / 10 + 2 * MS_TILE + 31) & ~31ull;
  if ((s = reserve(c->sort_tmp, (size_t)MS_BINS * ocap0 * 8))) return s;
  const MsBufs bf0{(const uint64_t *)in, (uint64_t *)out, (uint64_t *)c->sort_tmp.ptr, nullptr};
  std::vector<MsSeg> one{MsSeg{0, n, 0, 0}};
  std::vector<uint32_t> tiles;
  const uint32_t stile = (c->opt[NUT_OPT_SORT_BD] == 512 ? 512u : (uint32_t)MS_THREADS) * MS_ITEMS * ms_halves();
  const uint64_t nt0 = tile_table(one, stile, tiles);
  if (nt0 > 0x7FFFFFFFull) return fail(NUT_ERR_UNSUPPORTED, "nut_sort_i64: too many tiles");
  std::vector<uint64_t> cur0(MS_BINS + 1, 0);
  for (int d = 0; d < MS_BINS; ++d) cur0[d] = (uint64_t)d * ocap0;
  s = ar.begin(MetaArena::align(sizeof(MsSeg)) + MetaArena::align(tiles.size() * 4) +
               MetaArena::align(cur0.size() * 8));
  if (s) return s;
  MsSeg *dseg;
  uint32_t *dtile;
  uint64_t *dcur0;
  if ((s = ar.upload(one, &dseg)) || (s = ar.upload(tiles, &dtile)) || (s = ar.upload(cur0, &dcur0))) return s;
  // the full 64-bit range maps to the keys' top digits: the shift digits (no range check,
  // fewer registers) do the same partition
  const bool ident = m0.base == 0 && m0.t == 32 && m0.mul == (1u << 18);
  unsigned long long *dc0 = (unsigned long long *)dcur0, *of0 = (unsigned long long *)(dcur0 + MS_BINS);
  if (ident)
    capped_scatter(c, nt0, bf0, dseg, dtile, MsDigit{0, 64 - MS_BITS, MS_BINS - 1}, flip, dc0, 2, ocap0, of0);
  else
    capped_scatter(c, nt0, bf0, dseg, dtile, m0, flip, dc0, 2, ocap0, of0);
  NUT_HIP(hipGetLastError());
  std::vector<uint64_t> end0(MS_BINS + 1);
  NUT_HIP(hipMemcpyAsync(end0.data(), dcur0, end0.size() * 8, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  if (end0[MS_BINS]) return NUT_ERR_CAPACITY;
  // ---- level 1: each region -> 512 capped regions of tmp2
  std::vector<MsSeg> segs(MS_BINS);
  std::vector<uint64_t> dbase(MS_BINS);
  uint64_t cmax = 0, run = 0;
  for (int d = 0; d < MS_BINS; ++d) {
    const uint64_t cnt = end0[d] - cur0[d];
    segs[d] = MsSeg{cur0[d], cnt, 2, 0};
    dbase[d] = run;
    run += cnt;
    cmax = std::max(cmax, cnt);
  }
  const uint64_t ocap1 = ((cmax / MS_BINS) * 23 / 20 + 64 + 1) & ~1ull;
  if ((s = reserve(c->sort_tmp2, (size_t)MS_BINS * MS_BINS * ocap1 * 8))) return s;
  const MsBufs bf{(const uint64_t *)in, (uint64_t *)out, (uint64_t *)c->sort_tmp.ptr, (uint64_t *)c->sort_tmp2.ptr};
  const uint64_t nt1 = tile_table(segs, stile, tiles);
  if (nt1 > 0x7FFFFFFFull) return fail(NUT_ERR_UNSUPPORTED, "nut_sort_i64: too many tiles");
  const uint64_t nr = (uint64_t)MS_BINS * MS_BINS, lcap = nr;
  std::vector<uint64_t> cur1(nr + 1, 0);
  for (uint64_t r = 0; r < nr; ++r) cur1[r] = r * ocap1;
  s = ar.begin(MetaArena::align(segs.size() * sizeof(MsSeg)) + MetaArena::align(tiles.size() * 4) +
               MetaArena::align(cur1.size() * 8) + MetaArena::align(dbase.size() * 8) +
               MetaArena::align(LS_NCLS * lcap * sizeof(MsSeg)) + LS_NCLS * MetaArena::align((lcap + 1) * 4) + 1024);
  if (s) return s;
  MsSeg *dsegs;
  uint32_t *dt1;
  uint64_t *dcur1, *ddb;
  if ((s = ar.upload(segs, &dsegs)) || (s = ar.upload(tiles, &dt1)) || (s = ar.upload(cur1, &dcur1)) ||
      (s = ar.upload(dbase, &ddb)))
    return s;
  MsSeg *lists = (MsSeg *)ar.alloc(LS_NCLS * lcap * sizeof(MsSeg));
  unsigned int *counts = (unsigned int *)ar.alloc(4 * LS_NCLS);
  uint32_t *fb[LS_NCLS];
  for (auto &f : fb) f = (uint32_t *)ar.alloc((lcap + 1) * 4);
  NUT_HIP(hipMemsetAsync(counts, 0, 4 * LS_NCLS, st));
  MsMap m1 = m0;
  m1.dshift = 0;
  m1.maxx = ~0ull;  // level 0 checked every key
  unsigned long long *dc1 = (unsigned long long *)dcur1, *of1 = (unsigned long long *)(dcur1 + nr);
  if (ident)
    capped_scatter(c, nt1, bf, dsegs, dt1, MsDigit{0, 64 - 2 * MS_BITS, MS_BINS - 1}, flip, dc1, 3, ocap1, of1);
  else
    capped_scatter(c, nt1, bf, dsegs, dt1, m1, flip, dc1, 3, ocap1, of1);
  hipLaunchKernelGGL(ms_plan_capped_kernel, dim3(MS_BINS), dim3(MS_BINS), 0, st, (const unsigned long long *)dcur1,
                     (const uint64_t *)ddb, ocap1, m0, lists, lcap, counts, (unsigned long long *)(dcur1 + nr));
  NUT_HIP(hipGetLastError());
  uint64_t *hc = c->host_pinned;
  static_assert(4 * LS_NCLS <= 16, "class counts in the first two pinned words");
  NUT_HIP(hipMemcpyAsync(hc, counts, 4 * LS_NCLS, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipMemcpyAsync(hc + 2, dcur1 + nr, 8, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  if (hc[2]) return NUT_ERR_CAPACITY;
  const uint32_t *cnt = (const uint32_t *)hc;
  uint32_t ncls[LS_NCLS];
  for (int k = 0; k < LS_NCLS; ++k) ncls[k] = cnt[k];
  for (int cls = LS_NCLS - 1; cls >= 0; --cls)
    if ((s = launch_local_dev(c, bf, flip, lists + (uint64_t)cls * lcap, ncls[cls], fb[cls], cls))) return s;
  c->sort_bytes = 48 * n;
  c->sort_levels = 2;
  return NUT_OK;
}

nut_status msd_sort_i64(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n, uint64_t flip,
                        const uint64_t *bounds) {
  hipStream_t st = c->stream;
  c->sort_bytes = 0;
  c->sort_levels = 0;
  c->timer.begin(st, NUT_KERNEL_SORT);
  if (n >= kCappedMin) {
    nut_status s = msd_sort_capped(c, in, out, n, flip, bounds);
    if (s != NUT_ERR_CAPACITY) {
      c->timer.end(st);
      if (!s) NUT_HIP(hipStreamSynchronize(st));
      return s;
    }
    c->sort_bytes = 0;  // a skewed distribution: the exact layout below
    c->sort_levels = 0;
  }
  nut_status s = c->sort_tmp.reserve(n * 8);
  if (s) {
    c->timer.end(st);
    return s;
  }
  const MsBufs bf{(const uint64_t *)in, (uint64_t *)out, (uint64_t *)c->sort_tmp.ptr, nullptr};
  MetaArena ar{c};

  if (n <= LS_CAP) {  // one workgroup, all 64 bits
    std::vector<MsSeg> one{{0, n, 0, 64}};
    s = ar.begin(1024);
    if (s) return s;
    s = launch_local(c, ar, bf, flip, one, ls_class(n));
    if (s) return s;
    c->sort_bytes = 16 * n;
    c->timer.end(st);
    return NUT_OK;
  }

  // Levels of MS_BITS-bit digits of (key - base), most significant first.  The first
  // histogram speculates base 0 and the top 9 key bits while it reduces the keys' min and
  // max; if the top bits barely vary (a narrow key range, e.g. a sample-sort rank's), the
  // histogram is redone with base = min and the digit below the top bit of max - min.
  std::vector<MsSeg> big{{0, n, 0, 0}}, scat, next, small[LS_NCLS], done;
  std::vector<uint32_t> tiles;
  std::vector<uint64_t> hist, cursor;
  MsDigit dg{0, 64 - MS_BITS, (uint32_t)MS_BINS - 1};
  bool first = true;
  while (!big.empty()) {
    // ---- histograms of the level's digit over the big segments
    const uint64_t nht = tile_table(big, MH_HTILE, tiles);
    if (nht > 0x7FFFFFFFull) return fail(NUT_ERR_UNSUPPORTED, "nut_sort_i64: too many tiles");
    const size_t hbytes = big.size() * MS_BINS * 8;
    s = ar.begin(MetaArena::align(big.size() * sizeof(MsSeg)) + MetaArena::align(tiles.size() * 4) +
                 MetaArena::align(hbytes) + 256);
    if (s) return s;
    MsSeg *dseg;
    uint32_t *dtile;
    if ((s = ar.upload(big, &dseg)) || (s = ar.upload(tiles, &dtile))) return s;
    unsigned long long *dhist = (unsigned long long *)ar.alloc(hbytes);
    unsigned long long *dmm = (unsigned long long *)ar.alloc(16);
    NUT_HIP(hipMemsetAsync(dhist, 0, hbytes, st));
    if (first) {
      const unsigned long long init[2] = {~0ull, 0ull};
      ar.keep.emplace_back((const char *)init, (const char *)init + 16);
      NUT_HIP(hipMemcpyAsync(dmm, ar.keep.back().data(), 16, hipMemcpyHostToDevice, st));
    }
    for (const MsSeg &sg : big) c->sort_bytes += 8 * sg.count;
    hipLaunchKernelGGL(ms_hist_kernel<MsDigit>, dim3((unsigned)nht), dim3(MH_THREADS), 0, st, bf, (const MsSeg *)dseg,
                       (const uint32_t *)dtile, dg, flip, dhist, first ? dmm : nullptr);
    NUT_HIP(hipGetLastError());
    hist.resize(big.size() * MS_BINS);
    NUT_HIP(hipMemcpyAsync(hist.data(), dhist, hbytes, hipMemcpyDeviceToHost, st));
    unsigned long long hmm[2] = {0, 0};
    if (first) NUT_HIP(hipMemcpyAsync(hmm, dmm, 16, hipMemcpyDeviceToHost, st));
    NUT_HIP(hipStreamSynchronize(st));
    if (first) {
      first = false;
      const uint64_t mn = hmm[0], mx = hmm[1];
      if (mn == mx) {  // all keys equal
        done.push_back(MsSeg{0, n, 0, 0});
        big.clear();
        break;
      }
      if ((mx >> (64 - MS_BITS)) - (mn >> (64 - MS_BITS)) < (uint64_t)MS_BINS / 4) {
        const int hb = 64 - __builtin_clzll(mx - mn);  // (key - mn) < 2^hb
        const int w = std::min(MS_BITS, hb);
        dg = MsDigit{mn, hb - w, (1u << w) - 1u};
        continue;
      }
    }
    const int hi = dg.shift;  // sub-segments of this level agree on bits >= shift
    // ---- classify: segments whose digit takes one value pass through unmoved
    scat.clear();
    next.clear();
    std::vector<uint64_t> scat_hist;
    auto classify = [&](MsSeg sg) {
      if (hi == 0) {
        done.push_back(sg);
      } else if (sg.count <= LS_CAP) {
        sg.aux = (uint32_t)hi;
        sg.base = dg.base;
        small[ls_class(sg.count)].push_back(sg);
      } else {
        next.push_back(sg);
      }
    };
    for (size_t i = 0; i < big.size(); ++i) {
      const uint64_t *h = &hist[i * MS_BINS];
      int nz = 0;
      for (int d = 0; d < MS_BINS; ++d) nz += h[d] != 0;
      if (nz <= 1) {
        classify(big[i]);
      } else {
        scat.push_back(big[i]);
        scat_hist.insert(scat_hist.end(), h, h + MS_BINS);
      }
    }
    if (!scat.empty()) {
      // ---- scatter level
      cursor.resize(scat.size() * MS_BINS);
      for (size_t i = 0; i < scat.size(); ++i) {
        uint64_t run = scat[i].start;
        const uint32_t nb = scat[i].buf == 2 ? 1u : 2u;
        for (int d = 0; d < MS_BINS; ++d) {
          const uint64_t cnt = scat_hist[i * MS_BINS + d];
          cursor[i * MS_BINS + d] = run;
          if (cnt) classify(MsSeg{run, cnt, nb, 0});
          run += cnt;
        }
      }
      const uint64_t nst = tile_table(scat, MS_TILE * ms_halves(), tiles);
      if (nst > 0x7FFFFFFFull) return fail(NUT_ERR_UNSUPPORTED, "nut_sort_i64: too many tiles");
      s = ar.begin(MetaArena::align(scat.size() * sizeof(MsSeg)) + MetaArena::align(tiles.size() * 4) +
                   MetaArena::align(cursor.size() * 8));
      if (s) return s;
      MsSeg *dsc;
      uint32_t *dt;
      uint64_t *dcur;
      if ((s = ar.upload(scat, &dsc)) || (s = ar.upload(tiles, &dt)) || (s = ar.upload(cursor, &dcur))) return s;
      for (const MsSeg &sg : scat) c->sort_bytes += 16 * sg.count;
      ++c->sort_levels;
      const unsigned sgrid = (unsigned)std::min<uint64_t>(nst, (uint64_t)c->num_cus);  // persistent, 1 per CU (128 KB LDS)
      launch_scatter(st, sgrid, bf, (const MsSeg *)dsc, (const uint32_t *)dt, (uint32_t)nst, dg, flip,
                     (unsigned long long *)dcur);
      NUT_HIP(hipGetLastError());
    }
    big.swap(next);
    const int w = std::min(MS_BITS, hi);  // the next level's digit: the bits just below
    dg = MsDigit{dg.base, hi - w, (1u << w) - 1u};
    break;  // further levels are planned on the device
  }
  // ---- further levels: device-planned (histogram, cursors and class lists on the GPU)
  for (std::vector<MsSeg> over; !big.empty(); big.swap(over)) {
    if (dg.mask == 0) {  // the previous level consumed the last bit: each segment is one key value
      done.insert(done.end(), big.begin(), big.end());
      break;
    }
    if ((s = device_level(c, ar, bf, dg, flip, big, over))) return s;
    const int hi = dg.shift, w = std::min(MS_BITS, hi);
    dg = MsDigit{dg.base, hi - w, (1u << w) - 1u};
  }
  // ---- finish: local sorts and equal-key runs
  size_t total = 256;
  for (auto &v : small) total += MetaArena::align(v.size() * sizeof(MsSeg)) + MetaArena::align((v.size() + 1) * 4);
  std::vector<uint32_t> ctiles;
  const uint64_t nct = tile_table(done, MH_TILE, ctiles);
  total += MetaArena::align(done.size() * sizeof(MsSeg)) + MetaArena::align(ctiles.size() * 4);
  s = ar.begin(total);
  if (s) return s;
  for (int cls = LS_NCLS - 1; cls >= 0; --cls) {
    for (const MsSeg &sg : small[cls]) c->sort_bytes += 16 * sg.count;
    if ((s = launch_local(c, ar, bf, flip, small[cls], cls))) return s;
  }
  for (const MsSeg &sg : done) c->sort_bytes += 16 * sg.count;
  if (!done.empty()) {
    MsSeg *dd;
    uint32_t *dt;
    if ((s = ar.upload(done, &dd)) || (s = ar.upload(ctiles, &dt))) return s;
    hipLaunchKernelGGL(ms_copy_kernel, dim3((unsigned)nct), dim3(MH_THREADS), 0, st, bf, (const MsSeg *)dd,
                       (const uint32_t *)dt, flip);
    NUT_HIP(hipGetLastError());
  }
  c->timer.end(st);
  NUT_HIP(hipStreamSynchronize(st));  // host tables in `ar.keep` must outlive the copies
  return NUT_OK;
}

// Unstable range partition for the sample sort (dist.cpp sort_member): out holds bucket 0's
// keys, then bucket 1's, ...; counts_host[b] = bucket b's count.  A 512-bin histogram pass
// and one scatter level of the MSD sort's kernels (24 B/key; the stable LSD-pass partition,
// nut_partition_i64, took a look-back chain per tile) — the keys of one bucket may come out
// in any order: the receiver sorts them, and an equal-key bucket split over ranks by
// position is split among equal keys.
nut_status partition_i64_ranges(nut_ctx *c, const int64_t *in, uint64_t n, const int64_t *spl, int ns, int64_t *out,
                                uint64_t *counts_host) {
  if (ns < 0 || ns > 63) return fail(NUT_ERR_INVALID_ARG, "partition_i64_ranges: 0..63 splitters");
  for (int b = 0; b <= ns; ++b) counts_host[b] = 0;
  if (n == 0) return NUT_OK;
  DeviceGuard g(c->device);
  hipStream_t st = c->stream;
  MsSplit dg;
  dg.ns = ns;
  dg.sbits = 0;
  while ((ns + 1) << (dg.sbits + 1) <= MS_BINS) ++dg.sbits;
  for (int j = 0; j < 63; ++j) dg.e[j] = j < ns ? spl[j] : INT64_MAX;
  // cell c holds the flipped keys [c << 52, (c + 1) << 52): its first bucket, and whether
  // a splitter lies inside it
  std::vector<uint8_t> tab(MsSplit::kAux);
  for (int cc = 0, j = 0; cc < MsSplit::kAux; ++cc) {
    const uint64_t lo = (uint64_t)cc << 52, hi = lo + ((1ull << 52) - 1);
    while (j < ns && ((uint64_t)spl[j] ^ 0x8000000000000000ull) <= lo) ++j;
    int j2 = j;
    while (j2 < ns && ((uint64_t)spl[j2] ^ 0x8000000000000000ull) <= hi) ++j2;
    tab[cc] = (uint8_t)(j | (j2 > j ? 0x80 : 0));
  }
  const MsBufs bf{(const uint64_t *)in, (uint64_t *)out, nullptr, nullptr};
  std::vector<MsSeg> one{MsSeg{0, n, 0, 0}};
  std::vector<uint32_t> htiles, stiles;
  std::vector<MsSeg> sone = one;
  const uint64_t nht = tile_table(one, MH_HTILE, htiles);
  const uint64_t nst = tile_table(sone, MS_TILE * ms_halves(), stiles);
  if (nht > 0x7FFFFFFFull || nst > 0x7FFFFFFFull) return fail(NUT_ERR_UNSUPPORTED, "partition_i64_ranges: too many tiles");
  MetaArena ar{c};
  nut_status s = ar.begin(2 * MetaArena::align(sizeof(MsSeg)) + MetaArena::align(htiles.size() * 4) +
                          MetaArena::align(stiles.size() * 4) + 2 * MetaArena::align(MS_BINS * 8) +
                          MetaArena::align(MsSplit::kAux));
  if (s) return s;
  MsSeg *dseg, *dsseg;
  uint32_t *dht, *dst;
  uint8_t *dtab;
  if ((s = ar.upload(one, &dseg)) || (s = ar.upload(htiles, &dht)) || (s = ar.upload(sone, &dsseg)) ||
      (s = ar.upload(stiles, &dst)) || (s = ar.upload(tab, &dtab)))
    return s;
  dg.tab = dtab;
  unsigned long long *dhist = (unsigned long long *)ar.alloc(MS_BINS * 8);
  unsigned long long *dcur = (unsigned long long *)ar.alloc(MS_BINS * 8);
  c->timer.begin(st, NUT_KERNEL_SORT);
  NUT_HIP(hipMemsetAsync(dhist, 0, MS_BINS * 8, st));
  hipLaunchKernelGGL(ms_hist_kernel<MsSplit>, dim3((unsigned)nht), dim3(MH_THREADS), 0, st, bf, (const MsSeg *)dseg,
                     (const uint32_t *)dht, dg, (uint64_t)0, dhist, (unsigned long long *)nullptr);
  NUT_HIP(hipGetLastError());
  uint64_t *hc = c->host_pinned;  // 512 words = the whole 4 KB staging buffer
  NUT_HIP(hipMemcpyAsync(hc, dhist, MS_BINS * 8, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  std::vector<uint64_t> cur(MS_BINS, 0);
  uint64_t run = 0;
  for (int d = 0; d < ((ns + 1) << dg.sbits); ++d) {
    counts_host[d >> dg.sbits] += hc[d];
    cur[d] = run;
    run += hc[d];
  }
  if (run != n) {
    c->timer.end(st);
    return fail(NUT_ERR_UNSUPPORTED, "partition_i64_ranges: histogram lost keys");
  }
  ar.keep.emplace_back((const char *)cur.data(), (const char *)(cur.data() + MS_BINS));
  NUT_HIP(hipMemcpyAsync(dcur, ar.keep.back().data(), MS_BINS * 8, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL((ms_scatter_kernel<ms_halves(), MsSplit>), dim3((unsigned)std::min<uint64_t>(nst, (uint64_t)c->num_cus)),
                     dim3(MS_THREADS), 0, st, bf, (const MsSeg *)dsseg, (const uint32_t *)dst, (uint32_t)nst, dg,
                     (uint64_t)0, dcur, 1, (uint64_t)0, (unsigned long long *)nullptr);
  NUT_HIP(hipGetLastError());
  c->timer.end(st);
  NUT_HIP(hipStreamSynchronize(st));  // the host tables of `ar` live until here
  return NUT_OK;
}

#endif  // NUT_MSD_KERNELS_ONLY

}  // namespace nut
