// agg_kernel.hpp — the streaming filter -> group-by -> aggregate kernel.
//
//   * grid-stride over row pairs; each lane holds FOUR rows per step (two 16-B loads per
//     column) and the loads of the NEXT step are issued before the current step is
//     folded (register double buffer), so a wave keeps HBM requests in flight while it
//     computes — the Q1 kernel runs at 8 waves/CU (private accumulators take the LDS);
//   * per-workgroup hash table in LDS; the home of a key is a 2-slot bucket read with one
//     ds_read_b128, so most rows resolve without entering the probe loop;
//   * keys are found lock-free; NEW keys of tables that publish more than the slot word
//     (two-key tuples, private ids) are inserted under a block-level LDS lock, so nothing
//     is half-published and nothing is wasted; single-key shared tables claim by CAS;
//   * PRIV: the first P groups of a block fold into per-thread private accumulators
//     laid out [group][agg][thread] (plain read-modify-write, conflict-free), reduced
//     once per block; keys in a small range (one key < 256, or two keys < 16 each:
//     dictionary codes such as Q1's flags) find their private id in a direct map (one LDS
//     word per key value, filled from the hash table on first sight) without hashing;
//   * rows of keys the block table does not admit fold into the global table (g_row);
//     at block end the LDS table is merged into the global (HBM) table.
#pragma once

#include "agg_ops.hpp"

namespace nut {

// ------------------------------------------------------------------ LDS table
// Layout (dynamic LDS, this order, 16-B aligned):
//   slot[cap+1] u64 | agg[na][cap+1] u64 | k12[cap+1] {i64,i64} (NK=2) | did[cap+1] u32
//   (PRIV) | dslot[kPrivMax] u32 + dmap[kDirect] u32 (PRIV) | ctl[4] u32 | priv[P][na][BD] u64 (PRIV)
enum { CTL_CLAIMED = 0, CTL_SPECIAL = 1, CTL_LOCK = 2, CTL_NDENSE = 3 };
constexpr uint32_t kNoDense = 0xFFFFFFFFu;
constexpr uint32_t kDirect = 256;  // direct-map entries (PRIV): key < 256, or 16 x 16 key pairs

struct LTable {
  uint64_t *slot, *agg;
  i64x2 *k12;
  uint32_t *did, *dslot, *ctl;
  uint32_t *dmap;  // PRIV: private id of a small key (tuple), kNoDense until first seen
  uint64_t *priv;
  uint32_t *spill;  // spill mode: the block's append cursor (LDS)
  uint32_t *shist;  //   and its histogram of the key hash's top byte (LDS, 256)
};

__host__ __device__ inline size_t lds_layout(uint32_t cap, int nk, int na, bool privm, int P, int bd,
                                             size_t *o_k12, size_t *o_did, size_t *o_dslot, size_t *o_ctl,
                                             size_t *o_priv) {
  const size_t stride = cap + 1;
  size_t o = stride * 8 * (1 + (size_t)na);
  o = (o + 15) & ~size_t(15);
  *o_k12 = o;
  if (nk == 2) o += stride * 16;
  *o_did = o;
  if (privm) o += stride * 4;
  *o_dslot = o;
  if (privm) o += (kPrivMax + kDirect) * 4;
  *o_ctl = o;
  o += 16;
  o = (o + 15) & ~size_t(15);
  *o_priv = o;
  if (privm) o += (size_t)P * na * bd * 8;
  return (o + 15) & ~size_t(15);
}

// slot word of a key: the key itself (one key) or a 64-bit hash nudged off the empty
// marker (two keys; the tuple is verified against k12)
template <int NK>
__device__ __forceinline__ uint64_t lkey(uint64_t k1, uint64_t k2) {
  if (NK == 1) return k1;
  uint64_t h = k1 * kGolden ^ ((k2 + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full);
  h ^= h >> 29;
  return h == kEmpty ? h ^ 1ull : h;
}
// home bucket (4 slots, 32-B aligned) of a slot word
constexpr uint32_t kBucket = 4;
// on-chip table home: Fibonacci hash of the xor-folded key (3 VALU ops; the table has
// at most 2^15 slots, so 32 product bits are plenty)
__device__ __forceinline__ uint32_t lhome(uint64_t w, int log2cap) {
  const uint32_t f = (uint32_t)w ^ (uint32_t)(w >> 32);
  return ((f * 0x9E3779B1u) >> (32 - log2cap)) & ~(kBucket - 1);
}

// direct-map index of a key (tuple), or kDirect when it is out of the map's range
template <int NK>
__device__ __forceinline__ uint32_t direct_idx(uint64_t k1, uint64_t k2) {
  if (NK == 1) return k1 < kDirect ? (uint32_t)k1 : kDirect;
  return (k1 | k2) < 16 ? (uint32_t)(k1 << 4 | k2) : kDirect;
}

template <int NK>
__device__ __forceinline__ bool keys_match(const LTable &t, uint32_t s, uint64_t k1, uint64_t k2) {
  if (NK == 1) return true;
  const i64x2 kk = t.k12[s];
  return (uint64_t)kk.x == k1 && (uint64_t)kk.y == k2;
}

// Lock-free walk from the home bucket: slot index, or -1 (reached an empty slot, at
// `empty_at`) or -2 (chain exhausted).
template <int NK>
__device__ __forceinline__ int32_t l_walk(const LTable &t, uint32_t cap, int log2cap, uint64_t w, uint64_t k1,
                                          uint64_t k2, uint32_t &empty_at) {
  uint32_t s = lhome(w, log2cap);
  for (uint32_t probe = 0; probe < cap; ++probe) {
    const uint64_t cur = __hip_atomic_load(&t.slot[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == w && keys_match<NK>(t, s, k1, k2)) return (int32_t)s;
    if (cur == kEmpty) {
      empty_at = s;
      return -1;
    }
    s = (s + 1) & (cap - 1);
  }
  return -2;
}

// Slow path of the lookup (home bucket missed): find or insert; returns the slot (>= 0)
// or -1 (not admitted: the row goes to the global table).
template <int NK, bool LOCKED>
__device__ __noinline__ int32_t l_find_slow(const LTable t, const uint32_t cap, const uint32_t limit,
                                            const int log2cap, const int priv, const uint64_t w, const uint64_t k1,
                                            const uint64_t k2) {
  if (NK == 1 && w == kEmpty) {
    t.ctl[CTL_SPECIAL] = 1u;
    return (int32_t)cap;
  }
  uint32_t e = 0;
  int32_t s = l_walk<NK>(t, cap, log2cap, w, k1, k2, e);
  if (s >= 0) return s;
  if (s == -2) return -1;
  if (!LOCKED) {
    // claim by CAS along the chain from the first empty slot
    for (uint32_t probe = 0; probe < cap; ++probe) {
      uint64_t cur = t.slot[e];
      if (cur == w) return (int32_t)e;
      if (cur == kEmpty) {
        if (*(volatile uint32_t *)&t.ctl[CTL_CLAIMED] >= limit) return -1;
        cur = atomicCAS((unsigned long long *)&t.slot[e], (unsigned long long)kEmpty, (unsigned long long)w);
        if (cur == kEmpty) {
          atomicAdd(&t.ctl[CTL_CLAIMED], 1u);
          return (int32_t)e;
        }
        if (cur == w) return (int32_t)e;
      }
      e = (e + 1) & (cap - 1);
    }
    return -1;
  }
  // Locked insert.  Every waiting lane of the wave retries until it has run its own
  // critical section; the lock holder's section runs in the same pass (no SIMT
  // deadlock); other waves retry.  The slot word is published last (release).
  int32_t res = -1;
  bool done = false;
  for (uint32_t spins = 0;; ++spins) {
    if (!done) {
      if (__hip_atomic_exchange(&t.ctl[CTL_LOCK], 1u, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
        uint32_t e2 = 0;
        res = l_walk<NK>(t, cap, log2cap, w, k1, k2, e2);
        if (res == -1) {
          if (t.ctl[CTL_CLAIMED] < limit) {
            if (NK == 2) t.k12[e2] = i64x2{(int64_t)k1, (int64_t)k2};
            if (t.did) {
              uint32_t d = t.ctl[CTL_NDENSE];
              if (d < (uint32_t)priv) {
                t.dslot[d] = e2;
                t.ctl[CTL_NDENSE] = d + 1;
              } else {
                d = kNoDense;
              }
              t.did[e2] = d;
            }
            t.ctl[CTL_CLAIMED] += 1u;
            __hip_atomic_store(&t.slot[e2], w, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            res = (int32_t)e2;
          }
        } else if (res == -2) {
          res = -1;
        }
        __hip_atomic_store(&t.ctl[CTL_LOCK], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        done = true;
      }
    }
    if (__all(done) || spins > (1u << 20)) break;
    __builtin_amdgcn_s_sleep(1);
  }
  return done ? res : -1;
}

// ------------------------------------------------------------------ row loads
template <class S>
struct Rows {
  uint64_t k1[4], k2[4];
  uint64_t pv[S::MP > 0 ? S::MP : 1][4];
  uint64_t vv[S::MV > 0 ? S::MV : 1][4];
};

// computed keys of a generated shape (bit j: key j is S::key(), nut_agg_spec.key_prog)
template <class S>
__device__ constexpr int key_prog_mask() {
  if constexpr (S::kProg) return S::kKeyProg;
  else return 0;
}

// VEC: 1 = all columns 16-B aligned (vector loads), 0 = decided at run time (p.vec)
template <int VEC>
__device__ __forceinline__ void load2(const AggArgs &p, const uint64_t *col, uint64_t i, uint64_t &x, uint64_t &y) {
  if (VEC == 1 || p.vec) {
    // non-temporal: the columns stream through once (measured A/B on one box: config 3
    // 2.98 -> 2.63 ms, Q1 7.95 -> 7.42 ms)
    const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(col + i));
    x = v.x;
    y = v.y;
  } else {
    x = col[i];
    y = col[i + 1];
  }
}

// rows {i0, i0+1, i1, i1+1}; TAIL: guard every row against n
template <int NK, class S, int VEC, bool TAIL>
__device__ __forceinline__ void load_rows(const AggArgs &p, uint64_t i0, uint64_t i1, uint64_t nend, Rows<S> &x) {
  auto ld = [&](const uint64_t *col, uint64_t (&d)[4]) {
    if (TAIL) {
      d[0] = i0 < nend ? col[i0] : 0;
      d[1] = i0 + 1 < nend ? col[i0 + 1] : 0;
      d[2] = i1 < nend ? col[i1] : 0;
      d[3] = i1 + 1 < nend ? col[i1 + 1] : 0;
    } else {
      load2<VEC>(p, col, i0, d[0], d[1]);
      load2<VEC>(p, col, i1, d[2], d[3]);
    }
  };
#pragma unroll
  for (int t = 0; t < S::MP; ++t)
    if (t < S::np(p)) ld(p.pred_col[t], x.pv[t]);
  constexpr int KP = key_prog_mask<S>();
  if (NK == 1 && p.nokey) {
#pragma unroll
    for (int r = 0; r < 4; ++r) x.k1[r] = 0;
  } else if (!(KP & 1)) {
    ld(p.keys[0], x.k1);
  }
  if (NK == 2 && !(KP & 2)) ld(p.keys[1], x.k2);
#pragma unroll
  for (int c = 0; c < S::MV; ++c)
    if (c < S::nv(p)) ld(p.val_col[c], x.vv[c]);
}

// ------------------------------------------------------------------ spill (partitioned mode)
// Append the rows with sl[r] == -1 to the staged arrays: one cursor atomic per wave and
// row slot, on the block's LDS cursor.  A value a masked-out row does not give its aggregate is staged as the
// aggregate's identity (f64 SUM: -0.0, which leaves every sum bit-identical), a COUNT as
// 1 / 0 (the partition pass then sums it).
template <int NK, class S>
__device__ __forceinline__ void spill_rows(const AggArgs &p, const LTable &lt, const uint64_t (&kk1)[4],
                                           const uint64_t (&kk2)[4], const int32_t (&sl)[4],
                                           const uint64_t (&av)[S::MA][4],
                                           const bool (&vm)[S::MA][4]) {
  const int lane = threadIdx.x & 63;
  const uint64_t region = (uint64_t)blockIdx.x * p.sp_region;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool mine = sl[r] == -1;
    const uint64_t m = __ballot(mine);
    if (!m) continue;
    const int leader = __builtin_ctzll(m);
    uint32_t b = 0;
    if (lane == leader) b = atomicAdd(lt.spill, (uint32_t)__popcll(m));
    b = __shfl(b, leader, 64);
    if (mine) {
      const uint64_t pos = region + b + lane_rank(m);
      const uint64_t k1 = kk1[r], k2 = NK == 2 ? kk2[r] : 0;
      atomicAdd(&lt.shist[owner_hash(k1, k2, NK) >> 56], 1u);
      p.sp_cols[1][pos] = k1;
      if (NK == 2) p.sp_cols[2][pos] = k2;
#pragma unroll
      for (int a = 0; a < S::MA; ++a) {
        if (a < S::na(p) && p.sp_map[a] >= 0) {
          const int k = S::kind(p, a);
          uint64_t v = av[a][r];
          if (k == AK_COUNT) v = vm[a][r] ? 1ull : 0ull;
          else if (!vm[a][r])
            v = k == AK_SUM_F64 ? 0x8000000000000000ull
                                : (k == AK_MIN_F64 || k == AK_MAX_F64) ? ord_to_f64(agg_init(k)) : agg_init(k);
          p.sp_cols[3 + p.sp_map[a]][pos] = v;
        }
      }
    }
  }
}

// ------------------------------------------------------------------ fold four rows
template <int NK, bool PRIV, int BD, class S, bool TAIL>
__device__ __forceinline__ void consume_rows(const AggArgs &p, const LTable &lt, uint64_t i0, uint64_t i1,
                                             uint64_t nend, const Rows<S> &x, bool &err) {
  constexpr int R = 4;
  constexpr bool LOCKED = NK == 2 || PRIV;
  bool ok[R];
#pragma unroll
  for (int r = 0; r < R; ++r) ok[r] = !TAIL || ((r < 2 ? i0 : i1) + (r & 1)) < nend;
  uint64_t kk1[R], kk2[R];
#pragma unroll
  for (int r = 0; r < R; ++r) kk1[r] = x.k1[r], kk2[r] = NK == 2 ? x.k2[r] : 0;
  if constexpr (S::kProg) {
    // generated WHERE program (padding rows of the tail never raise)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      bool e = false;
      const bool w = S::where(p, x.vv, r, e);
      err = err || (e && ok[r]);
      ok[r] = ok[r] && w;
    }
    // computed keys: their errors count for rows passing WHERE
    constexpr int KP = key_prog_mask<S>();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      bool e = false;
      if (KP & 1) kk1[r] = S::key(p, 0, x.vv, r, e);
      if (NK == 2 && (KP & 2)) kk2[r] = S::key(p, 1, x.vv, r, e);
      err = err || (e && ok[r]);
    }
  }
  // WHERE: one decision per term per four rows
#pragma unroll
  for (int t = 0; t < S::MP; ++t) {
    if (t < S::np(p)) {
      const int op = S::pop(p, t);
      if (op >= NUT_IN) {
        // [NOT] IN: uniform loop over the set (scalar loads), one compare per value
        const int ns = p.pred_nset[t];
        const bool f64 = S::ptype(p, t) == NUT_T_F64;
        bool in[R] = {};
        for (int i = 0; i < ns; ++i) {
          const uint64_t sv = p.pred_set[t][i];
#pragma unroll
          for (int r = 0; r < R; ++r)
            in[r] = in[r] || (f64 ? as_f64(x.pv[t][r]) == as_f64(sv) : x.pv[t][r] == sv);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) ok[r] = ok[r] && (in[r] == (op == NUT_IN));
      } else {
        const uint64_t k = p.pred_k[t];
        with_pred(S::ptype(p, t), op, [&](auto OPC, auto TYC) {
          constexpr int OP = decltype(OPC)::value, TY = decltype(TYC)::value;
#pragma unroll
          for (int r = 0; r < R; ++r) ok[r] = ok[r] && pred1<OP, TY>(x.pv[t][r], k);
        });
      }
    }
  }
  // GROUP BY.  PRIV: keys in the direct map's range take their private id from it (one
  // LDS word, no hashing); the rest — and every row of a shared table — do a home-bucket
  // lookup of all four rows (four ds_read_b128 in flight), then the probe loop only for
  // rows that missed.  A wave none of whose rows needs the table skips it.
  const uint32_t cap = p.lds_cap;
  int32_t sl[R];
  bool need[R];
  uint32_t di[R], dm[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    sl[r] = -2;
    need[r] = ok[r];
    di[r] = kDirect;
    dm[r] = kNoDense;
  }
  if (PRIV && cap) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      di[r] = direct_idx<NK>(kk1[r], kk2[r]);
      dm[r] = di[r] < kDirect ? lt.dmap[di[r]] : kNoDense;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (ok[r] && dm[r] != kNoDense) sl[r] = 0, need[r] = false;  // any slot >= 0: the fold goes private
    }
  }
  if (cap) {
    bool any = false;
#pragma unroll
    for (int r = 0; r < R; ++r) any = any || need[r];
    if (!PRIV || __any(any)) {
      uint64_t w[R];
      u64x2 b0[R], b1[R];
      uint32_t hb[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        w[r] = lkey<NK>(kk1[r], kk2[r]);
        hb[r] = lhome(w[r], p.lds_log2);
        b0[r] = *reinterpret_cast<const u64x2 *>(&lt.slot[hb[r]]);
        b1[r] = *reinterpret_cast<const u64x2 *>(&lt.slot[hb[r] + 2]);
      }
      if (LOCKED) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (need[r]) {
          // home bucket: the first slot holding w; no match and an empty slot in the
          // bucket ends the chain (no deletes: a key never sits behind an empty slot)
          int32_t s = -1;
          const uint64_t c[4] = {b0[r].x, b0[r].y, b1[r].x, b1[r].y};
#pragma unroll
          for (int j = 3; j >= 0; --j) s = c[j] == w[r] ? (int32_t)hb[r] + j : s;
          bool end = (c[0] == kEmpty) | (c[1] == kEmpty) | (c[2] == kEmpty) | (c[3] == kEmpty);
          if (NK == 2 && s >= 0 && !keys_match<NK>(lt, (uint32_t)s, kk1[r], kk2[r])) s = -1, end = false;
          if (NK == 1 && w[r] == kEmpty) s = -1, end = true;
          if (s < 0 && !end) {
            // continue the probe chain past the bucket (inline: a few slots at most)
            uint32_t e = (hb[r] + kBucket) & (cap - 1);
            for (uint32_t probe = kBucket; probe < cap; ++probe) {
              const uint64_t cur =
                  LOCKED ? __hip_atomic_load(&lt.slot[e], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) : lt.slot[e];
              if (cur == w[r] && keys_match<NK>(lt, e, kk1[r], kk2[r])) {
                s = (int32_t)e;
                break;
              }
              if (cur == kEmpty) break;
              e = (e + 1) & (cap - 1);
            }
          }
          // not present: insert (or find a concurrent insert) out of line
          if (s < 0) s = l_find_slow<NK, LOCKED>(lt, cap, p.lds_limit, p.lds_log2, p.priv, w[r], kk1[r], kk2[r]);
          sl[r] = s;
        }
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) sl[r] = ok[r] ? -1 : -2;
  }
  uint32_t dd[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (!PRIV) {
      dd[r] = kNoDense;
    } else if (!need[r]) {
      dd[r] = dm[r];  // a direct-map hit (or a row WHERE dropped: sl = -2, never folded)
    } else {
      dd[r] = (sl[r] >= 0 && sl[r] < (int32_t)cap) ? lt.did[sl[r]] : kNoDense;
      // the private id of a slot never changes once published: cache it for the key
      if (dd[r] != kNoDense && di[r] < kDirect) lt.dmap[di[r]] = dd[r];
    }
  }

  // aggregate inputs
  uint64_t av[S::MA][R];
  bool vm[S::MA][R];  // row mask per aggregate (expression shapes; constant true otherwise)
#pragma unroll
  for (int a = 0; a < S::MA; ++a) {
#pragma unroll
    for (int r = 0; r < R; ++r) av[a][r] = 0, vm[a][r] = true;
    if constexpr (S::kProg) {
      // errors count only for rows the aggregate actually takes
#pragma unroll
      for (int r = 0; r < R; ++r) {
        bool em = false, ev = false;
        vm[a][r] = S::valid(p, a, x.vv, r, em);
        if (S::kind(p, a) != AK_COUNT) av[a][r] = S::value(p, a, x.vv, r, ev);
        err = err || (ok[r] && (em || (vm[a][r] && ev)));
      }
    } else if (a < S::na(p) && S::kind(p, a) != AK_COUNT) {
      const int a0 = S::arg(p, a, 0), a1 = S::arg(p, a, 1), a2 = S::arg(p, a, 2);
      with_expr(S::expr(p, a), [&](auto EC) {
        constexpr int E = decltype(EC)::value;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          auto pick = [&](int c) {
            uint64_t v = x.vv[0][r];
#pragma unroll
            for (int q = 1; q < S::MV; ++q) v = c == q ? x.vv[q][r] : v;
            return v;
          };
          av[a][r] = eval<E>(pick(a0), pick(a1), pick(a2));
        }
      });
    }
  }
  // fold
  const uint32_t stride = cap + 1;
#pragma unroll
  for (int a = 0; a < S::MA; ++a) {
    if (a < S::na(p)) {
      with_kind(S::kind(p, a), [&](auto KC) {
        constexpr int K = decltype(KC)::value;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (sl[r] >= 0 && vm[a][r]) {
            if (PRIV && dd[r] != kNoDense) {
              uint64_t *pw = &lt.priv[((size_t)dd[r] * S::na(p) + a) * BD + threadIdx.x];
              *pw = fold<K>(*pw, av[a][r]);
            } else {
              fold_atomic<K>(&lt.agg[a * stride + sl[r]], av[a][r]);
            }
          }
        }
      });
    }
  }
  // rows the block table did not admit
  if (p.sp_counts) {
    spill_rows<NK, S>(p, lt, kk1, kk2, sl, av, vm);
    return;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (sl[r] == -1 && NK == 1 && p.dense) {
      atomicOr(&p.gt->ctl[1], 4u);  // dense mode needs every group on chip: the host reruns hashed
    } else if (sl[r] == -1) {
      uint64_t g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      uint32_t m = 0;
#pragma unroll
      for (int a = 0; a < S::MA && a < 8; ++a) g[a] = av[a][r], m |= vm[a][r] ? 1u << a : 0u;
      g_row<NK>(p.gt, (int64_t)kk1[r], (int64_t)kk2[r], m, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7]);
    }
  }
}

// ------------------------------------------------------------------ the kernel
template <int NK, bool PRIV, int BD, class S, int VEC>
__global__ __launch_bounds__(BD) void agg_kernel(AggArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const uint32_t cap = p.lds_cap;
  const uint32_t stride = cap + 1;
  const int na = S::na(p);
  LTable lt;
  {
    size_t o_k12, o_did, o_dslot, o_ctl, o_priv;
    lds_layout(cap, NK, na, PRIV, p.priv, BD, &o_k12, &o_did, &o_dslot, &o_ctl, &o_priv);
    char *b = (char *)smem;
    lt.slot = (uint64_t *)b;
    lt.agg = lt.slot + stride;
    lt.k12 = (i64x2 *)(b + o_k12);
    lt.did = PRIV ? (uint32_t *)(b + o_did) : nullptr;
    lt.dslot = (uint32_t *)(b + o_dslot);
    lt.dmap = PRIV ? lt.dslot + kPrivMax : nullptr;
    lt.ctl = (uint32_t *)(b + o_ctl);
    lt.priv = (uint64_t *)(b + o_priv);
  }
  __shared__ uint32_t s_spill;
  __shared__ uint32_t s_shist[256];
  lt.spill = &s_spill;
  lt.shist = s_shist;
  if (p.sp_counts) {
    if (threadIdx.x == 0) s_spill = 0;
    for (int i = threadIdx.x; i < 256; i += BD) s_shist[i] = 0;
    __syncthreads();
  }
  if (cap) {
    for (uint32_t s = threadIdx.x; s < stride; s += BD) {
      lt.slot[s] = kEmpty;
#pragma unroll
      for (int a = 0; a < S::MA; ++a)
        if (a < na) lt.agg[a * stride + s] = agg_init(S::kind(p, a));
      if (PRIV) lt.did[s] = kNoDense;
    }
    if (threadIdx.x < 4) lt.ctl[threadIdx.x] = 0;
    if (PRIV)
      for (uint32_t i = threadIdx.x; i < kDirect; i += BD) lt.dmap[i] = kNoDense;
    if (PRIV) {
#pragma unroll
      for (int a = 0; a < S::MA; ++a)
        if (a < na) {
          const uint64_t init = agg_init(S::kind(p, a));
          for (int d = 0; d < p.priv; ++d) lt.priv[((size_t)d * na + a) * BD + threadIdx.x] = init;
        }
    }
    __syncthreads();
  }

  // grid-stride over row pairs; a step takes pairs q and q + gstride (four rows) and
  // the next step's loads are issued before this step is folded.  Segment mode: this
  // block's rows [seg_off[2b], seg_off[2b+1]), block-stride (row base `rb`).
  uint64_t rb = 0, nrows = p.n, gstride = (uint64_t)gridDim.x * BD, q = (uint64_t)blockIdx.x * BD + threadIdx.x;
  if (p.seg_off) {
    rb = p.seg_end ? p.seg_off[blockIdx.x] : p.seg_off[2 * blockIdx.x];
    nrows = (p.seg_end ? (p.seg_cut ? min(p.seg_end[blockIdx.x], p.seg_cut[blockIdx.x]) : p.seg_end[blockIdx.x])
                       : p.seg_off[2 * blockIdx.x + 1]) -
            rb;
    gstride = BD;
    q = threadIdx.x;
  }
  const uint64_t nend = rb + nrows;
  const uint64_t npairs = (nrows + 1) / 2;
  const uint64_t full_pairs = nrows / 2;
  bool err = false;  // an expression raised (integer division by zero)
  if (q + gstride < full_pairs) {
    Rows<S> cur;
    load_rows<NK, S, VEC, false>(p, rb + 2 * q, rb + 2 * (q + gstride), nend, cur);
    for (;;) {
      const uint64_t qn = q + 2 * gstride;
      const bool more = qn + gstride < full_pairs;
      // shared-table kernels: unconditional (the last step reloads this one, unused) — a
      // load under `if (more)` was issued where its data is consumed, a step late, no
      // prefetch at all (same-box A/B: G = 1000 2.81 -> 2.73 ms).  The private-accumulator
      // kernels (Q1, expression shapes) keep the late load: their 6 waves per CU hide it,
      // and the prefetch's registers cost them (Q1 7.74 -> 7.80, Q12 8.72 -> 8.90 ms)
      Rows<S> nxt;
      if (!PRIV) {
        const uint64_t ql = more ? qn : q;
        load_rows<NK, S, VEC, false>(p, rb + 2 * ql, rb + 2 * (ql + gstride), nend, nxt);
      } else if (more) {
        load_rows<NK, S, VEC, false>(p, rb + 2 * qn, rb + 2 * (qn + gstride), nend, nxt);
      }
      consume_rows<NK, PRIV, BD, S, false>(p, lt, rb + 2 * q, rb + 2 * (q + gstride), nend, cur, err);
      q = qn;
      if (!more) break;
      cur = nxt;
    }
  }
  if (q < npairs) {  // last partial step: at most two pairs left for this lane
    const uint64_t q1 = q + gstride < npairs ? q + gstride : q;
    Rows<S> x;
    load_rows<NK, S, VEC, true>(p, rb + 2 * q, rb + 2 * q1, nend, x);
    // a duplicate second pair (q1 == q) is masked out by placing it past the end
    consume_rows<NK, PRIV, BD, S, true>(p, lt, rb + 2 * q, q1 == q ? nend : rb + 2 * q1, nend, x, err);
  }

  if constexpr (S::kProg) {
    if (err) atomicOr(&p.gt->ctl[1], 2u);  // flag 2: division by zero (query fails)
  }
  if (p.sp_counts) {
    __syncthreads();
    if (threadIdx.x == 0) p.sp_counts[blockIdx.x] = s_spill;
    for (int i = threadIdx.x; i < 256; i += BD)
      if (s_shist[i]) atomicAdd(&p.sp_hist[i], (unsigned long long)s_shist[i]);
  }
  if (!cap) return;
  __syncthreads();
  if (PRIV) {
    // reduce each (group, aggregate) column of the private accumulators: 8 threads per
    // column, fixed order, then one LDS atomic merge into the shared slot
    const uint32_t nd = min(lt.ctl[CTL_NDENSE], (uint32_t)p.priv);
    const int part = threadIdx.x & 7;
    for (uint32_t pi = threadIdx.x >> 3; pi < nd * (uint32_t)na; pi += BD / 8) {
      const uint32_t d = pi / na, a = pi % na;
      const uint64_t *col = &lt.priv[(size_t)pi * BD];
#pragma unroll
      for (int aa = 0; aa < S::MA; ++aa) {
        if ((int)a == aa) {
          with_kind(S::kind(p, aa), [&](auto KC) {
            constexpr int K = decltype(KC)::value;
            uint64_t acc = col[part];
            for (int j = part + 8; j < BD; j += 8) acc = combine<K>(acc, col[j]);
#pragma unroll
            for (int off = 4; off >= 1; off >>= 1) acc = combine<K>(acc, __shfl_xor(acc, off, 8));
            if (part == 0) agg_merge_word(&lt.agg[aa * stride + lt.dslot[d]], K, acc);
          });
        }
      }
    }
    __syncthreads();
  }
  // merge the block's table into the global table
  const GTable t = *p.gt;
  const uint64_t gstr = t.cap + 1;
  if (NK == 1 && p.dense && p.dcount) {
    // dense staging: the block's region of the table, its count for the ordering pass
    __shared__ uint32_t s_m;
    if (threadIdx.x == 0) s_m = 0;
    __syncthreads();
    const uint64_t base = (p.dbase + blockIdx.x) * p.dregion;
    for (uint32_t s = threadIdx.x; s < stride; s += BD) {
      const uint64_t wd = lt.slot[s];
      const bool occ = s < cap ? wd != kEmpty : lt.ctl[CTL_SPECIAL] != 0u;
      const uint64_t m = __ballot(occ);
      uint32_t r = 0;
      if (m) {
        const int leader = __builtin_ctzll(m);
        uint32_t b = 0;
        if ((threadIdx.x & 63) == (uint32_t)leader) b = atomicAdd(&s_m, (uint32_t)__popcll(m));
        r = __shfl(b, leader, 64) + lane_rank(m);
      }
      if (!occ) continue;
      t.slot[base + r] = s < cap ? wd : kEmpty;
#pragma unroll
      for (int a = 0; a < S::MA; ++a)
        if (a < na) t.agg[a * gstr + base + r] = lt.agg[a * stride + s];
    }
    __syncthreads();
    if (threadIdx.x == 0) p.dcount[blockIdx.x] = s_m;
    return;
  }
  if (NK == 1 && p.dense) {
    // the partition's groups are complete and no other block holds them: append them at
    // slots claimed with one global atomic per block (no probing, no atomic merges); the
    // table is a plain array afterwards (nut_groups.dense)
    __shared__ uint32_t s_n;
    __shared__ uint64_t s_base;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    for (uint32_t s = threadIdx.x; s < cap; s += BD) {
      const uint64_t m = __ballot(lt.slot[s] != kEmpty);
      if (m && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(m)) atomicAdd(&s_n, (uint32_t)__popcll(m));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t b = s_n ? atomicAdd(&t.shard[0], s_n) : 0;
      if (b + s_n > t.limit) atomicOr(&t.ctl[1], 1u);  // more groups than the table holds: retried larger
      s_base = b + s_n > t.limit ? ~0ull : b;
      s_n = 0;
    }
    __syncthreads();
    const uint64_t base = s_base;
    for (uint32_t s = threadIdx.x; s < stride; s += BD) {
      const uint64_t wd = lt.slot[s];
      const bool occ = s < cap ? wd != kEmpty : lt.ctl[CTL_SPECIAL] != 0u;
      const uint64_t m = __ballot(occ && s < cap);
      uint32_t r = 0;
      if (m) {
        const int leader = __builtin_ctzll(m);
        uint32_t b = 0;
        if ((threadIdx.x & 63) == (uint32_t)leader) b = atomicAdd(&s_n, (uint32_t)__popcll(m));
        r = __shfl(b, leader, 64) + lane_rank(m);
      }
      if (!occ) continue;
      if (s == cap) {  // the empty-marker key: its dedicated slot, merged as usual
        const int64_t gs = g_find<1>(t, key_hash<1>((int64_t)kEmpty, 0), (int64_t)kEmpty, 0);
#pragma unroll
        for (int a = 0; a < S::MA; ++a)
          if (a < na) agg_merge_word(&t.agg[a * gstr + gs], S::kind(p, a), lt.agg[a * stride + s]);
        continue;
      }
      if (base == ~0ull) continue;
      const uint64_t pos = base + r;
      t.slot[pos] = wd;
#pragma unroll
      for (int a = 0; a < S::MA; ++a)
        if (a < na) t.agg[a * gstr + pos] = lt.agg[a * stride + s];
    }
    return;
  }
  for (uint32_t s = threadIdx.x; s < stride; s += BD) {
    const uint64_t wd = lt.slot[s];
    const bool occ = s < cap ? wd != kEmpty : lt.ctl[CTL_SPECIAL] != 0u;
    if (!occ) continue;
    const int64_t k1 = NK == 1 ? (int64_t)(s < cap ? wd : kEmpty) : lt.k12[s].x;
    const int64_t k2 = NK == 1 ? 0 : lt.k12[s].y;
    const int64_t gs = g_find<NK>(t, key_hash<NK>(k1, k2), k1, k2);
    if (gs < 0) continue;
#pragma unroll
    for (int a = 0; a < S::MA; ++a)
      if (a < na) agg_merge_word(&t.agg[a * gstr + gs], S::kind(p, a), lt.agg[a * stride + s]);
  }
}

}  // namespace nut
