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
//   * level histograms (ms_hist_kernel): one 256-bin LDS histogram per 64 Ki-key tile of a
//     segment, flushed with 256 global atomics; the first also reduces OR / AND of all keys,
//     whose XOR names the digits that vary (the others are skipped everywhere).
//   * scatter levels (ms_scatter_kernel): keys only, so a level needs no stability — the
//     local sort re-sorts every segment completely.  A tile (8192 keys) ranks its keys with
//     LDS atomics (one per key, no ballots), stages them in LDS in digit order and claims
//     each digit's output run with ONE global atomic on the segment's digit cursor: no
//     look-back chain, no spin, progress independent of dispatch order.
//   * local sort (ms_local_kernel): a segment of <= 32768 keys is loaded into registers
//     (lo / hi 32-bit halves), sorted by its remaining varying digits with stable LSD passes
//     entirely in LDS (ballot peer ranking, per-wave digit counters, exchange by halves so
//     the exchange buffer is 4 B/key = 128 KiB), and written once, coalesced.
// Keys map to u64 with the sign bit flipped (DESC: its complement) on the first load and
// back on the final store.
#include <algorithm>
#include <vector>

#include "common.hpp"
#include "sort.hpp"

namespace nut {

constexpr int MH_THREADS = 256;
constexpr uint32_t MH_TILE = 1u << 16;  // keys per histogram / copy tile
constexpr int MS_THREADS = 512;
constexpr int MS_ITEMS = 16;
constexpr uint32_t MS_TILE = MS_THREADS * MS_ITEMS;  // 8192 keys per scatter tile
constexpr int MS_BINS = 256;
// local-sort classes: threads x max items per thread (ms_local_kernel)
constexpr int LS_S_THREADS = 256, LS_S_ITEMS = 8;    // <= 2048 keys
constexpr int LS_M_THREADS = 512, LS_M_ITEMS = 16;   // <= 8192 keys
constexpr int LS_L_THREADS = 1024, LS_L_ITEMS = 24;  // <= 24576 keys
constexpr uint64_t LS_S_CAP = LS_S_THREADS * LS_S_ITEMS;
constexpr uint64_t LS_M_CAP = LS_M_THREADS * LS_M_ITEMS;
constexpr uint64_t LS_CAP = LS_L_THREADS * LS_L_ITEMS;

// A contiguous run [start, start + count) of one of the three buffers.
struct MsSeg {
  uint64_t start, count;
  uint32_t buf;  // 0: caller's input (raw int64: flip on load), 1: out, 2: tmp
  uint32_t aux;  // hist / scatter / copy: first tile of the segment; local sort: digits left
};
struct MsBufs {
  const uint64_t *in;
  uint64_t *a;  // out
  uint64_t *b;  // tmp
};
struct MsShifts {
  int s[8];  // bit offsets of the varying digits, least significant first
};

__device__ __forceinline__ const uint64_t *ms_src(const MsBufs &bf, uint32_t buf) {
  return buf == 0 ? bf.in : (buf == 1 ? bf.a : bf.b);
}

// ---------------------------------------------------------------- level histogram
__global__ __launch_bounds__(MH_THREADS) void ms_hist_kernel(MsBufs bf, const MsSeg *__restrict__ segs,
                                                             const uint32_t *__restrict__ tile_seg, int shift,
                                                             uint64_t flip, unsigned long long *__restrict__ hist,
                                                             unsigned long long *__restrict__ orand) {
  __shared__ uint32_t h[MS_BINS];
  const int tid = threadIdx.x;
  h[tid] = 0;
  __syncthreads();
  const uint32_t s = tile_seg[blockIdx.x];
  const MsSeg sg = segs[s];
  const uint64_t lo = (uint64_t)(blockIdx.x - sg.aux) * MH_TILE;
  const uint32_t cnt = (uint32_t)min<uint64_t>(MH_TILE, sg.count - lo);
  const uint64_t *src = ms_src(bf, sg.buf) + sg.start + lo;
  const uint64_t f = sg.buf == 0 ? flip : 0;
  uint64_t vor = 0, vand = ~0ull;
  for (uint32_t i = tid; i < cnt; i += MH_THREADS * 8) {
    uint64_t k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t idx = i + j * MH_THREADS;
      k[j] = idx < cnt ? (__builtin_nontemporal_load(src + idx) ^ f) : 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (i + j * MH_THREADS < cnt) {
        atomicAdd(&h[(k[j] >> shift) & 255], 1u);
        vor |= k[j];
        vand &= k[j];
      }
    }
  }
  if (orand) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      vor |= __shfl_xor(vor, off, 64);
      vand &= __shfl_xor(vand, off, 64);
    }
    if ((tid & 63) == 0) {
      atomicOr(&orand[0], (unsigned long long)vor);
      atomicAnd(&orand[1], (unsigned long long)vand);
    }
  }
  __syncthreads();
  if (h[tid]) atomicAdd(&hist[(uint64_t)s * MS_BINS + tid], (unsigned long long)h[tid]);
}

// ---------------------------------------------------------------- scatter level
// Unstable partition of every listed segment by digit (key >> shift) & 255 into the other
// buffer (in / tmp -> ... see ms_dst).  cursor[s][d] starts at the absolute position of
// sub-segment (s, d) and is advanced by one atomic per (tile, digit).
__device__ __forceinline__ uint64_t *ms_dst(const MsBufs &bf, uint32_t buf) { return buf == 2 ? bf.a : bf.b; }

// Persistent: workgroup b takes tiles b, b + grid, ...; the next tile's keys are loaded into
// the key registers as soon as the current tile is staged in LDS, so its HBM latency hides
// behind the current tile's write-out (and the segment lookup behind the ranking).
__global__ __launch_bounds__(MS_THREADS, 4) void ms_scatter_kernel(MsBufs bf, const MsSeg *__restrict__ segs,
                                                                   const uint32_t *__restrict__ tile_seg, uint32_t ntiles,
                                                                int shift, uint64_t flip,
                                                                unsigned long long *__restrict__ cursor) {
  __shared__ uint64_t s_keys[MS_TILE];
  __shared__ uint32_t s_cnt[MS_BINS];
  __shared__ uint32_t s_tex[MS_BINS];
  __shared__ uint64_t s_gb[MS_BINS];
  __shared__ uint32_t s_wsum[MS_BINS / kWave];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t t = blockIdx.x;
  uint64_t key[MS_ITEMS];
  auto load = [&](uint32_t tt, const MsSeg &g) {
    const uint64_t lo = (uint64_t)(tt - g.aux) * MS_TILE;
    const uint32_t cn = (uint32_t)min<uint64_t>(MS_TILE, g.count - lo);
    const uint64_t *sp = ms_src(bf, g.buf) + g.start + lo;
    const uint64_t ff = g.buf == 0 ? flip : 0;
#pragma unroll
    for (int i = 0; i < MS_ITEMS; ++i) {
      const uint32_t idx = (uint32_t)i * MS_THREADS + tid;
      key[i] = idx < cn ? (__builtin_nontemporal_load(sp + idx) ^ ff) : 0;
    }
  };
  uint32_t s = tile_seg[t];
  MsSeg sg = segs[s];
  load(t, sg);
  for (;;) {
    const uint64_t lo = (uint64_t)(t - sg.aux) * MS_TILE;
    const uint32_t cnt = (uint32_t)min<uint64_t>(MS_TILE, sg.count - lo);
    uint64_t *dst = ms_dst(bf, sg.buf);
    const uint32_t next = t + gridDim.x;
    const uint32_t ns = next < ntiles ? tile_seg[next] : 0;
    if (tid < MS_BINS) s_cnt[tid] = 0;
    __syncthreads();
    uint32_t rk[MS_ITEMS / 2];  // ranks in the tile's digit run (< 8192), 16-bit pairs
#pragma unroll
    for (int i = 0; i < MS_ITEMS; i += 2) rk[i / 2] = 0;
#pragma unroll
    for (int i = 0; i < MS_ITEMS; ++i) {
      const uint32_t idx = (uint32_t)i * MS_THREADS + tid;
      if (idx < cnt) rk[i / 2] |= atomicAdd(&s_cnt[(key[i] >> shift) & 255], 1u) << (16 * (i & 1));
    }
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
      s_gb[tid] = gb - tex;  // out position of LDS slot j of this digit = s_gb[d] + j
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MS_ITEMS; ++i) {
      const uint32_t idx = (uint32_t)i * MS_THREADS + tid;
      if (idx < cnt) s_keys[s_tex[(key[i] >> shift) & 255] + ((rk[i / 2] >> (16 * (i & 1))) & 0xFFFFu)] = key[i];
    }
    MsSeg nsg = sg;
    if (next < ntiles) {  // the key registers are free: fetch the next tile now
      nsg = segs[ns];
      load(next, nsg);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MS_ITEMS; ++i) {
      const uint32_t j = (uint32_t)i * MS_THREADS + tid;
      if (j < cnt) {
        const uint64_t k = s_keys[j];
        dst[s_gb[(k >> shift) & 255] + j] = k;
      }
    }
    if (next >= ntiles) break;
    __syncthreads();  // s_keys / s_gb are reused
    t = next;
    s = ns;
    sg = nsg;
  }
}

// ---------------------------------------------------------------- local sort
// One workgroup sorts one segment of <= THREADS * MAXK keys by its `aux` remaining varying
// digits (sh.s[0 .. aux-1], least significant first) and writes it to out at the same range.
//
// Main path (MSD split + bitonic windows):
//   1. the keys sit in registers; each takes a rank in its bucket with one LDS atomic, the
//      bucket being the top log2(THREADS) remaining varying bits (unstable: keys only);
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

template <int THREADS, int MAXK>
struct LocalCfg {
  static constexpr int WAVES = THREADS / kWave;
  static constexpr int CAP = THREADS * MAXK;
  static constexpr int LDS_KEYS = CAP < 16384 ? CAP : 16384;  // 8-B keys per round
  static constexpr int SB = CAP > 8192 ? 12 : (CAP > 2048 ? 11 : 9);  // bucket bits: ~4-6 keys each
  static constexpr int NB = 1 << SB;
  static constexpr int BPT = NB / THREADS;  // buckets per thread in the scan
  static_assert(BPT * THREADS == NB && BPT <= 4, "whole buckets per thread");
  static_assert(CAP <= 2 * LDS_KEYS, "at most two rounds");
  static constexpr int WPT = (CAP / LS_WS + THREADS - 1) / THREADS;  // windows per thread
  static_assert(WPT <= 2, "at most two windows per thread");
  // LDS: one round of 8-B keys, bucket counts -> starts, window starts, scan words
  static constexpr int NWIN = CAP / LS_WS + 2;  // window table entries (+ end)
  static constexpr int BYTES = LDS_KEYS * 8 + ((NB + 1) + NWIN + 16 + 2) * 4;
};

// block-wide exclusive scan of one value per thread (THREADS <= 1024); returns the prefix
// and writes the total to *total.  `ws` = 16 words of LDS.
template <int THREADS>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t *ws, uint32_t *total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
// exchange is v_cmp_lt_u64 + 4 v_cndmask (N = 16: 63 of them)
template <int N>
__device__ __forceinline__ void lane_sort(uint64_t (&v)[N]) {
  constexpr auto &net = OemTable<N>::net;
#pragma unroll
  for (int i = 0; i < net.n; ++i) {
    const uint64_t x = v[net.a[i]], y = v[net.b[i]];
    const bool lt = x < y;
    v[net.a[i]] = lt ? x : y;
    v[net.b[i]] = lt ? y : x;
  }
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

template <int THREADS, int MAXK>
__global__ __launch_bounds__(THREADS) void ms_local_kernel(MsBufs bf, const MsSeg *__restrict__ segs, MsShifts sh,
                                                           uint64_t flip, uint32_t *__restrict__ fb) {
  using C = LocalCfg<THREADS, MAXK>;
  constexpr int WAVES = C::WAVES, NB = C::NB, SB = C::SB;
  __shared__ __attribute__((aligned(16))) char lds[C::BYTES];
  uint64_t *s_keys = (uint64_t *)lds;
  uint32_t *s_off = (uint32_t *)(lds + C::LDS_KEYS * 8);  // [NB + 1] bucket counts -> starts, then c
  uint32_t *s_win = s_off + NB + 1;                        // [NWIN] window starts
  uint32_t *s_ws = s_win + C::NWIN;                        // 16 scan words
  uint32_t *s_misc = s_ws + 16;                            // [0] max window, [1] round split
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const MsSeg sg = segs[blockIdx.x];
  const uint32_t c = (uint32_t)sg.count;
  const int ndig = (int)sg.aux;
  const uint32_t K = (c + THREADS - 1) / THREADS;
  const uint32_t pw = (uint32_t)wave * kWave * K + lane;
  const uint64_t *src = ms_src(bf, sg.buf) + sg.start;
  uint64_t *dst = bf.a + sg.start;
  const uint64_t f = sg.buf == 0 ? flip : 0;
  uint64_t key[MAXK];
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    const uint32_t p = pw + (uint32_t)i * kWave;
    if ((uint32_t)i < K) key[i] = p < c ? (src[p] ^ f) : ~0ull;
  }
  if (ndig == 0) {  // every key equal: copy
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      const uint32_t p = pw + (uint32_t)i * kWave;
      if ((uint32_t)i < K && p < c) dst[p] = key[i] ^ flip;
    }
    return;
  }
  if (MS_STOP(1)) {
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < MAXK; ++i)
      if ((uint32_t)i < K) x ^= key[i];
    dst[tid] = x;
    return;
  }
  // ---- 1. bucket ranks: top SB remaining varying bits
  const int top = sh.s[ndig - 1];
  const int nxt = ndig >= 2 ? sh.s[ndig - 2] : -1;
  constexpr int EXTRA = SB - 8;
  auto bucket = [&](uint64_t k) -> uint32_t {
    uint32_t b = ((uint32_t)(k >> top) & 255u) << EXTRA;
    if (nxt >= 0) b |= (uint32_t)(k >> (nxt + 8 - EXTRA)) & ((1u << EXTRA) - 1u);
    return b;
  };
#pragma unroll
  for (int j = 0; j < C::BPT; ++j) s_off[C::BPT * tid + j] = 0;
  if (tid == 0) {
    s_misc[0] = 0;
    s_misc[1] = 0;
  }
  __syncthreads();
  uint32_t rk[(MAXK + 1) / 2];  // ranks in the bucket, 16-bit pairs
#pragma unroll
  for (int i = 0; i < MAXK; i += 2) rk[i / 2] = 0;
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    const uint32_t p = pw + (uint32_t)i * kWave;
    if ((uint32_t)i < K && p < c) rk[i / 2] |= atomicAdd(&s_off[bucket(key[i])], 1u) << (16 * (i & 1));
  }
  __syncthreads();
  // ---- 2. bucket starts (BPT consecutive buckets per thread) and windows
  {
    uint32_t cb[C::BPT], sum = 0;
#pragma unroll
    for (int j = 0; j < C::BPT; ++j) {
      cb[j] = s_off[C::BPT * tid + j];
      sum += cb[j];
    }
    uint32_t tot;
    uint32_t e = block_excl_scan<THREADS>(sum, s_ws, &tot);
    __syncthreads();  // every count read before the starts overwrite them
#pragma unroll
    for (int j = 0; j < C::BPT; ++j) {
      s_off[C::BPT * tid + j] = e;
      e += cb[j];
    }
    if (tid == 0) s_off[NB] = c;
  }
  __syncthreads();
  const uint32_t nq = (c + LS_WS - 1) / LS_WS;
#pragma unroll
  for (int j = 0; j < C::WPT; ++j) {
    const uint32_t q = (uint32_t)tid + (uint32_t)j * THREADS;
    if (q < nq) {  // first bucket start >= q * WS
      const uint32_t target = q * LS_WS;
      uint32_t lo = 0;
#pragma unroll
      for (int step = NB / 2; step >= 1; step >>= 1)
        if (s_off[lo + step - 1] < target) lo += step;
      s_win[q] = s_off[lo];  // s_off[NB] = c bounds the search
    }
  }
  if (tid == 0) s_win[nq] = c;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < C::WPT; ++j) {
    const uint32_t q = (uint32_t)tid + (uint32_t)j * THREADS;
    if (q < nq) {
      const uint32_t wa = s_win[q], wb = s_win[q + 1];
      atomicMax(&s_misc[0], wb - wa);
      if (wa <= (uint32_t)C::LDS_KEYS) atomicMax(&s_misc[1], q);
    }
  }
  __syncthreads();
  // rounds: windows [0, split) then [split, nq) with at most LDS_KEYS keys each
  const uint32_t split = c > (uint32_t)C::LDS_KEYS ? s_misc[1] : nq;
  const uint32_t mid = split < nq ? s_win[split] : c;
  if (s_misc[0] > (uint32_t)LS_MAX_WINDOW || c - mid > (uint32_t)C::LDS_KEYS) {
    if (tid == 0) fb[1 + atomicAdd(&fb[0], 1u)] = blockIdx.x;  // uniform: to ms_lsd_kernel
    return;
  }
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
  if (MS_STOP(3)) {
    __syncthreads();
    dst[tid] = s_keys[tid];
    return;
  }
  for (int round = 0; round < 2; ++round) {
    const uint32_t base = round ? mid : 0;
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
      const uint32_t wa = t < w1 ? s_win[t] - base : 0, wm = t < w1 ? s_win[t + 1] - s_win[t] : 0;
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
        uint32_t ga[8], gm[8];
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          const int l = mid32 ? __builtin_ctzll(mid32) : 0;
          gm[g] = mid32 ? __shfl(wm, l, 64) : 0;
          ga[g] = mid32 ? __shfl(wa, l, 64) : 0;
          mid32 &= mid32 - 1;
        }
        const uint32_t h = (uint32_t)lane & 31;
        uint64_t v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t mg = lane < 32 ? gm[2 * r] : gm[2 * r + 1], ag = lane < 32 ? ga[2 * r] : ga[2 * r + 1];
          v[r] = h < mg ? s_keys[ag + h] : ~0ull;
        }
        wave_bitonic32_multi<4>(v, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t mg = lane < 32 ? gm[2 * r] : gm[2 * r + 1], ag = lane < 32 ? ga[2 * r] : ga[2 * r + 1];
          if (h < mg) s_keys[ag + h] = v[r];
        }
      }
      for (uint64_t big = __ballot(wm > 32); big; big &= big - 1) {  // rare: one by one
        const int l = __builtin_ctzll(big);
        sort_window(s_keys + __shfl(wa, l, 64), __shfl(wm, l, 64), lane);
      }
    }
    __syncthreads();
    if (MS_STOP(4)) continue;
    const uint32_t rend = round ? c : mid;
    for (uint32_t j = tid; j < rend - base; j += THREADS) dst[base + j] = s_keys[j] ^ flip;
  }
}

// Fallback local sort: the segments ms_local_kernel listed in fb[1 ..] (fb[0] = count)
// get stable LSD passes in LDS.  Item i of lane l in wave w sits at canonical position
// w*64*K + i*64 + l; positions >= count hold all-ones padding, which a stable sort keeps
// behind every real key.
template <int THREADS, int MAXK>
__global__ __launch_bounds__(THREADS) void ms_lsd_kernel(MsBufs bf, const MsSeg *__restrict__ segs, MsShifts sh,
                                                         uint64_t flip, const uint32_t *__restrict__ fb) {
  using C = LocalCfg<THREADS, MAXK>;
  constexpr int WAVES = C::WAVES;
  if (blockIdx.x >= fb[0]) return;
  __shared__ uint32_t s_x[C::CAP];
  __shared__ uint32_t s_wcnt[WAVES][MS_BINS];
  __shared__ uint32_t s_tex[MS_BINS];
  __shared__ uint32_t s_wsum[MS_BINS / kWave];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const MsSeg sg = segs[fb[1 + blockIdx.x]];
  const uint32_t c = (uint32_t)sg.count;
  const int ndig = (int)sg.aux;
  const uint32_t K = (c + THREADS - 1) / THREADS;
  const uint32_t pw = (uint32_t)wave * kWave * K + lane;
  const uint64_t *src = ms_src(bf, sg.buf) + sg.start;
  uint64_t *dst = bf.a + sg.start;
  const uint64_t f = sg.buf == 0 ? flip : 0;
  uint32_t lo[MAXK], hi[MAXK], pos[MAXK];
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    if ((uint32_t)i < K) {
      const uint32_t p = pw + (uint32_t)i * kWave;
      const uint64_t k = p < c ? (src[p] ^ f) : ~0ull;
      lo[i] = (uint32_t)k;
      hi[i] = (uint32_t)(k >> 32);
    }
  }
  for (int pass = 0; pass < ndig; ++pass) {
    const int shift = sh.s[pass];
    const bool low = shift < 32;
    const int sft = low ? shift : shift - 32;
    for (int i = tid; i < WAVES * MS_BINS; i += THREADS) (&s_wcnt[0][0])[i] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      if ((uint32_t)i < K) {
        const uint32_t d = ((low ? lo[i] : hi[i]) >> sft) & 255u;
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
    if (tid < MS_BINS) {
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
    if (tid < MS_BINS) {
      uint32_t add = 0;
#pragma unroll
      for (int w = 0; w < MS_BINS / kWave; ++w) add += (w < wave) ? s_wsum[w] : 0u;
      s_tex[tid] = incl - tot + add;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MAXK; ++i) {
      if ((uint32_t)i < K) {
        const uint32_t d = ((low ? lo[i] : hi[i]) >> sft) & 255u;
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
    if ((uint32_t)i < K && p < c) dst[p] = (((uint64_t)hi[i] << 32) | lo[i]) ^ flip;
  }
}

// Segments whose keys are all equal (every varying digit consumed): out = key ^ flip.
__global__ __launch_bounds__(MH_THREADS) void ms_copy_kernel(MsBufs bf, const MsSeg *__restrict__ segs,
                                                             const uint32_t *__restrict__ tile_seg, uint64_t flip) {
  const MsSeg sg = segs[tile_seg[blockIdx.x]];
  const uint64_t lo = (uint64_t)(blockIdx.x - sg.aux) * MH_TILE;
  const uint32_t cnt = (uint32_t)min<uint64_t>(MH_TILE, sg.count - lo);
  const uint64_t *src = ms_src(bf, sg.buf) + sg.start + lo;
  uint64_t *dst = bf.a + sg.start + lo;
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
  nut_status begin(size_t total) {
    off = 0;
    if (total > c->sort_meta.bytes) {
      NUT_HIP(hipStreamSynchronize(c->stream));
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

template <int T, int K>
static void launch_class(hipStream_t st, const MsBufs &bf, const MsSeg *d, unsigned n, const MsShifts &sh,
                         uint64_t flip, uint32_t *fb) {
  hipLaunchKernelGGL((ms_local_kernel<T, K>), dim3(n), dim3(T), 0, st, bf, d, sh, flip, fb);
  hipLaunchKernelGGL((ms_lsd_kernel<T, K>), dim3(n), dim3(T), 0, st, bf, d, sh, flip, (const uint32_t *)fb);
}

static nut_status launch_local(nut_ctx *c, MetaArena &ar, const MsBufs &bf, const MsShifts &sh, uint64_t flip,
                               const std::vector<MsSeg> &segs, int cls) {
  if (segs.empty()) return NUT_OK;
  MsSeg *d;
  nut_status s = ar.upload(segs, &d);
  if (s) return s;
  uint32_t *fb = (uint32_t *)ar.alloc((segs.size() + 1) * 4);
  NUT_HIP(hipMemsetAsync(fb, 0, 4, c->stream));
  const unsigned n = (unsigned)segs.size();
  if (cls == 0)
    launch_class<LS_S_THREADS, LS_S_ITEMS>(c->stream, bf, d, n, sh, flip, fb);
  else if (cls == 1)
    launch_class<LS_M_THREADS, LS_M_ITEMS>(c->stream, bf, d, n, sh, flip, fb);
  else
    launch_class<LS_L_THREADS, LS_L_ITEMS>(c->stream, bf, d, n, sh, flip, fb);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

nut_status msd_sort_i64(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n, uint64_t flip) {
  hipStream_t st = c->stream;
  nut_status s = c->sort_tmp.reserve(n * 8);
  if (s) return s;
  const MsBufs bf{(const uint64_t *)in, (uint64_t *)out, (uint64_t *)c->sort_tmp.ptr};
  MetaArena ar{c};
  c->sort_bytes = 0;
  c->sort_levels = 0;
  c->timer.begin(st, NUT_KERNEL_SORT);

  if (n <= LS_CAP) {  // one workgroup, all eight digits
    MsShifts all;
    for (int p = 0; p < 8; ++p) all.s[p] = 8 * p;
    std::vector<MsSeg> one{{0, n, 0, 8}};
    s = ar.begin(1024);
    if (s) return s;
    s = launch_local(c, ar, bf, all, flip, one, n <= LS_S_CAP ? 0 : (n <= LS_M_CAP ? 1 : 2));
    if (s) return s;
    c->sort_bytes = 16 * n;
    c->timer.end(st);
    return NUT_OK;
  }

  std::vector<MsSeg> big{{0, n, 0, 0}}, scat, next, small[3], done;
  std::vector<uint32_t> tiles;
  std::vector<uint64_t> hist, cursor;
  std::vector<int> vary;  // varying digits, most significant first
  MsShifts asc{};         // varying digit shifts, least significant first
  int digit = 7;          // first histogram: digit 7, speculatively, with the OR/AND reduction
  bool first = true;
  while (!big.empty()) {
    // ---- histograms of `digit` over the big segments
    const uint64_t nht = tile_table(big, MH_TILE, tiles);
    if (nht > 0x7FFFFFFFull) return fail(NUT_ERR_UNSUPPORTED, "nut_sort_i64: too many tiles");
    const size_t hbytes = big.size() * MS_BINS * 8;
    s = ar.begin(MetaArena::align(big.size() * sizeof(MsSeg)) + MetaArena::align(tiles.size() * 4) +
                 MetaArena::align(hbytes) + 256);
    if (s) return s;
    MsSeg *dseg;
    uint32_t *dtile;
    if ((s = ar.upload(big, &dseg)) || (s = ar.upload(tiles, &dtile))) return s;
    unsigned long long *dhist = (unsigned long long *)ar.alloc(hbytes);
    unsigned long long *dor = (unsigned long long *)ar.alloc(16);
    NUT_HIP(hipMemsetAsync(dhist, 0, hbytes, st));
    if (first) {
      const unsigned long long init[2] = {0ull, ~0ull};
      ar.keep.emplace_back((const char *)init, (const char *)init + 16);
      NUT_HIP(hipMemcpyAsync(dor, ar.keep.back().data(), 16, hipMemcpyHostToDevice, st));
    }
    for (const MsSeg &sg : big) c->sort_bytes += 8 * sg.count;
    hipLaunchKernelGGL(ms_hist_kernel, dim3((unsigned)nht), dim3(MH_THREADS), 0, st, bf, (const MsSeg *)dseg,
                       (const uint32_t *)dtile, 8 * digit, flip, dhist, first ? dor : nullptr);
    NUT_HIP(hipGetLastError());
    hist.resize(big.size() * MS_BINS);
    NUT_HIP(hipMemcpyAsync(hist.data(), dhist, hbytes, hipMemcpyDeviceToHost, st));
    unsigned long long horand[2] = {0, 0};
    if (first) NUT_HIP(hipMemcpyAsync(horand, dor, 16, hipMemcpyDeviceToHost, st));
    NUT_HIP(hipStreamSynchronize(st));
    if (first) {
      first = false;
      const uint64_t diff = horand[0] ^ horand[1];
      for (int p = 7; p >= 0; --p)
        if ((diff >> (8 * p)) & 255) vary.push_back(p);
      for (size_t i = 0; i < vary.size(); ++i) asc.s[i] = 8 * vary[vary.size() - 1 - i];
      if (vary.empty()) {  // all keys equal
        MsSeg all{0, n, 0, 0};
        done.push_back(all);
        big.clear();
        break;
      }
      if (vary[0] != 7) {  // digit 7 constant: histogram the top varying digit instead
        digit = vary[0];
        continue;
      }
    }
    // varying digits below this level
    const int below = (int)(std::find(vary.begin(), vary.end(), digit) - vary.begin());
    const uint32_t left = (uint32_t)(vary.size() - 1 - below);
    // ---- classify: segments whose digit takes one value pass through unmoved
    scat.clear();
    next.clear();
    std::vector<uint64_t> scat_hist;
    auto classify = [&](MsSeg sg) {
      if (left == 0) {
        done.push_back(sg);
      } else if (sg.count <= LS_CAP) {
        sg.aux = left;
        small[sg.count <= LS_S_CAP ? 0 : (sg.count <= LS_M_CAP ? 1 : 2)].push_back(sg);
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
      const uint64_t nst = tile_table(scat, MS_TILE, tiles);
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
      const unsigned sgrid = (unsigned)std::min<uint64_t>(nst, (uint64_t)c->num_cus * 2);  // persistent, 2 per CU
      hipLaunchKernelGGL(ms_scatter_kernel, dim3(sgrid), dim3(MS_THREADS), 0, st, bf, (const MsSeg *)dsc,
                         (const uint32_t *)dt, (uint32_t)nst, 8 * digit, flip, (unsigned long long *)dcur);
      NUT_HIP(hipGetLastError());
    }
    big.swap(next);
    if (below + 1 < (int)vary.size()) digit = vary[below + 1];
  }
  // ---- finish: local sorts and equal-key runs
  size_t total = 256;
  for (auto &v : small) total += MetaArena::align(v.size() * sizeof(MsSeg)) + MetaArena::align((v.size() + 1) * 4);
  std::vector<uint32_t> ctiles;
  const uint64_t nct = tile_table(done, MH_TILE, ctiles);
  total += MetaArena::align(done.size() * sizeof(MsSeg)) + MetaArena::align(ctiles.size() * 4);
  s = ar.begin(total);
  if (s) return s;
  for (int cls = 2; cls >= 0; --cls) {
    for (const MsSeg &sg : small[cls]) c->sort_bytes += 16 * sg.count;
    if ((s = launch_local(c, ar, bf, asc, flip, small[cls], cls))) return s;
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

#endif  // NUT_MSD_KERNELS_ONLY

}  // namespace nut
