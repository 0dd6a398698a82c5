// aggregate.hip — host side of the fused  WHERE -> GROUP BY -> SUM/COUNT/MIN/MAX
// executor (BASELINE configs 3, 4): table lifecycle, kernel dispatch and the
// nut_groupby* / nut_groups_* / nut_q1 entry points of include/nutexec.h.
// Device code: agg_kernel.hpp + agg_ops.hpp (streaming kernel), gtable.hpp (global table).
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include "agg_kernel.hpp"
#include "gpart.hpp"
#include "fold.hpp"
#include "heavy.hpp"
#include "sort.hpp"
#include "jit.hpp"
#include "select_kernel.hpp"

// ============================================================== host side
using namespace nut;

struct nut_groups {
  nut_ctx *ctx = nullptr;
  int nk = 1, naggs = 0;
  int32_t kinds[NUT_MAX_AGGS] = {0};
  GTable gt{};                     // host copy of the descriptor
  GTable *dev_gt = nullptr;        // device copy (inside mem)
  void *mem = nullptr;             // table allocation
  size_t mem_bytes = 0;
  unsigned long long *dev_cursors = nullptr;  // [64] inside mem
  uint64_t *dev_segbase = nullptr;            // [2*64] inside mem
  bool dense = false;  // groups appended at slots 0.. (not at their hash): rehash before inserting
  // the table's control words as last read (read_ctl) while no launch has written the table
  // since: a result's size / to_host calls reuse them instead of one more round trip each
  uint32_t ctl_cache[4] = {0, 0, 0, 0};
  bool ctl_valid = false;
};

namespace {

int ilog2(uint64_t v) {
  int r = 0;
  while ((1ull << r) < v) ++r;
  return r;
}

uint32_t pack_kinds(const int32_t *k, int n) {
  uint32_t p = 0;
  for (int a = 0; a < n; ++a) p |= (uint32_t)(k[a] & 15) << (4 * a);
  return p;
}

nut_status validate(const nut_agg_spec *s) {
  if (!s) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: spec is NULL");
  if (s->nkeys < 0 || s->nkeys > 2) return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: 0, 1 or 2 key columns supported");
  if (s->npred < 0 || s->npred > NUT_MAX_PRED) return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: too many predicate terms");
  if (s->nvals < 0 || s->nvals > NUT_MAX_VALS) return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: too many value columns");
  if (s->naggs < 0 || s->naggs > NUT_MAX_AGGS) return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: too many aggregates");
  for (int k = 0; k < NUT_MAX_KEYS; ++k) {
    if (!s->key_prog[k].n) continue;
    if (!s->prog_mode) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: key programs need expression mode (prog_mode = 1)");
    if (k >= s->nkeys) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: key program past nkeys");
  }
  if (s->n) {
    for (int k = 0; k < s->nkeys; ++k)
      if (!s->keys[k] && !s->key_prog[k].n) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: NULL key column");
    for (int t = 0; t < s->npred; ++t) {
      if (!s->pred_col[t]) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: NULL predicate column");
      if (s->pred_op[t] < NUT_LT || s->pred_op[t] > NUT_NOT_IN) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad cmp op");
      if (s->pred_op[t] >= NUT_IN && (s->pred_nset[t] < 1 || s->pred_nset[t] > NUT_MAX_SET))
        return fail(NUT_ERR_INVALID_ARG, "nut_groupby: IN sets hold 1..16 values");
      if (s->pred_type[t] != NUT_T_I64 && s->pred_type[t] != NUT_T_F64)
        return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad predicate type");
    }
    for (int c = 0; c < s->nvals; ++c)
      if (!s->val_col[c]) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: NULL value column");
  }
  if (s->prog_mode) {
    if (s->npred || s->nvals) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: expression mode takes no pred_*/val_* terms");
    if (s->nprog_cols < 0 || s->nprog_cols > NUT_MAX_PROG_COLS)
      return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: expression programs read at most 16 columns");
    for (int c = 0; c < s->nprog_cols; ++c) {
      if (s->n && !s->prog_col[c]) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: NULL program column");
      if (s->prog_col_type[c] != NUT_T_I64 && s->prog_col_type[c] != NUT_T_F64)
        return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad program column type");
    }
    int32_t t;
    for (int k = 0; k < s->nkeys; ++k) {
      if (!s->key_prog[k].n) continue;
      nut_status st = prog_check(&s->key_prog[k], s->prog_col_type, s->nprog_cols, &t);
      if (st) return st;
      if (t == NUT_PT_F64) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: a key program is float64 (keys are int64)");
    }
    for (int a = 0; a < s->naggs; ++a) {
      int op = s->agg_op[a];
      if (op < NUT_AGG_SUM || op > NUT_AGG_MAX) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad aggregate op");
      if (op != NUT_AGG_COUNT) {
        nut_status st = prog_check(&s->agg_val[a], s->prog_col_type, s->nprog_cols, &t);
        if (st) return st;
      }
      if (s->agg_mask[a].n) {
        nut_status st = prog_check(&s->agg_mask[a], s->prog_col_type, s->nprog_cols, &t);
        if (st) return st;
      }
    }
    if (s->where.n) return prog_check(&s->where, s->prog_col_type, s->nprog_cols, &t);
    return NUT_OK;
  }
  for (int a = 0; a < s->naggs; ++a) {
    int op = s->agg_op[a];
    if (op < NUT_AGG_SUM || op > NUT_AGG_MAX) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad aggregate op");
    if (op == NUT_AGG_COUNT) continue;
    int e = s->agg_expr[a];
    if (e < NUT_EX_COL || e > NUT_EX_MUL_1M_1P) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: bad expression");
    int nargs = e == NUT_EX_COL ? 1 : e == NUT_EX_MUL_1M_1P ? 3 : 2;
    for (int j = 0; j < nargs; ++j) {
      int v = s->agg_arg[a][j];
      if (v < 0 || v >= s->nvals) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: expression argument out of range");
      if (e != NUT_EX_COL && s->val_type[v] != NUT_T_F64)
        return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: arithmetic expressions need f64 columns");
    }
  }
  return NUT_OK;
}

int32_t kind_of(const nut_agg_spec *s, int a) {
  int op = s->agg_op[a];
  if (op == NUT_AGG_COUNT) return AK_COUNT;
  bool i64 = s->agg_expr[a] == NUT_EX_COL && s->val_type[s->agg_arg[a][0]] == NUT_T_I64;
  if (s->prog_mode) {  // validated: the program type-checks
    int32_t t = NUT_PT_F64;
    (void)prog_check(&s->agg_val[a], s->prog_col_type, s->nprog_cols, &t);
    i64 = t != NUT_PT_F64;
  }
  switch (op) {
    case NUT_AGG_SUM: return i64 ? AK_SUM_I64 : AK_SUM_F64;
    case NUT_AGG_MIN: return i64 ? AK_MIN_I64 : AK_MIN_F64;
    default: return i64 ? AK_MAX_I64 : AK_MAX_F64;
  }
}

// LDS bytes of a table with `cap` slots (+1 special); two-key tables add a key arena
// of `cap` tuples (3/4 of it holds admitted keys, the rest absorbs lost claim races)
// (re)allocate the global table for `cap` slots and initialise it on the stream
nut_status alloc_table(nut_groups *g, uint64_t cap) {
  g->ctl_valid = false;
  const uint64_t stride = cap + 1;
  // two-key arena: one entry per claimable slot plus slack for claim races lost by
  // concurrent inserters of the same key (each loser leaks at most one entry)
  const uint64_t arena = g->nk == 2 ? cap + 65536 : 0;
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  size_t o_slot = carve(stride * 8);
  size_t o_agg = carve(stride * 8 * (size_t)std::max(g->naggs, 1));
  size_t o_a1 = carve(arena * 8 + 8);
  size_t o_a2 = carve(arena * 8 + 8);
  size_t o_ctl = carve(64);
  const int nsh_log2 = cap >= (1ull << 18) ? 8 : 0;
  const uint32_t nsh = 1u << nsh_log2;
  size_t o_sh = carve((size_t)nsh * 2 * 16 * 4);
  size_t o_gt = carve(sizeof(GTable));
  size_t o_cur = carve(64 * 8);
  size_t o_seg = carve(128 * 8);
  if (!(g->mem && g->mem_bytes >= off)) {
    if (g->mem) (void)hipFree(g->mem);
    g->mem = nullptr;
    nut_status ps = pool_take(g->ctx, off, &g->mem, &g->mem_bytes);  // a freed table's allocation, reused
    if (ps) return ps;
  }
  char *b = (char *)g->mem;
  GTable &t = g->gt;
  t.slot = (uint64_t *)(b + o_slot);
  t.agg = (uint64_t *)(b + o_agg);
  t.ak1 = (int64_t *)(b + o_a1);
  t.ak2 = (int64_t *)(b + o_a2);
  t.ctl = (uint32_t *)(b + o_ctl);
  t.shard = (uint32_t *)(b + o_sh);
  t.nsh_log2 = nsh_log2;
  t.cap = cap;
  t.log2cap = ilog2(cap);
  t.limit = (uint32_t)std::min<uint64_t>(cap - cap / 4, 0xFFFFFFF0ull);
  t.arena_cap = (uint32_t)std::min<uint64_t>(arena, 0xFFFFFFF0ull);
  // per shard: the claims of a uniformly hashed 1/nsh of the slots, +1/16 for variance
  t.limit_sh = nsh == 1 ? t.limit : t.limit / nsh + t.limit / nsh / 16;
  t.arena_sh = t.arena_cap / nsh;
  t.naggs = g->naggs;
  t.kinds = pack_kinds(g->kinds, g->naggs);
  g->dev_gt = (GTable *)(b + o_gt);
  g->dev_cursors = (unsigned long long *)(b + o_cur);
  g->dev_segbase = (uint64_t *)(b + o_seg);
  hipStream_t st = g->ctx->stream;
  NUT_HIP(hipMemsetAsync(t.ctl, 0, 64, st));
  NUT_HIP(hipMemsetAsync(t.shard, 0, (size_t)nsh * 2 * 16 * 4, st));
  NUT_HIP(hipMemcpyAsync(g->dev_gt, &g->gt, sizeof(GTable), hipMemcpyHostToDevice, st));
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)g->ctx->num_cus * 8);
  hipLaunchKernelGGL(gtable_init_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const GTable *)g->dev_gt, g->nk);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

nut_status read_ctl(nut_groups *g, uint32_t *ctl4) {
  if (g->ctl_valid) {
    memcpy(ctl4, g->ctl_cache, 16);
    return NUT_OK;
  }
  nut_ctx *c = g->ctx;
  hipLaunchKernelGGL(gtable_sum_kernel, dim3(1), dim3(256), 0, c->stream, (const GTable *)g->dev_gt);
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipMemcpyAsync(c->host_pinned, g->gt.ctl, 16, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  memcpy(ctl4, c->host_pinned, 16);
  memcpy(g->ctl_cache, ctl4, 16);
  g->ctl_valid = true;
  return NUT_OK;
}

// launch the streaming aggregation of spec's rows into g's table.  `kinds` are the
// per-row update kinds (COUNT partials are merged as integer sums).
// ---- kernel dispatch: compiled query shapes x {shared-only, private} x key count
using KernelFn = void (*)(AggArgs);
enum { SHAPE_GENERIC = 0, SHAPE_Q1, SHAPE_SUM, SHAPE_SUMCOUNT, SHAPE_ALL4 };

template <class S>
bool shape_matches(const nut_agg_spec *s, const int32_t *kinds, const AggArgs &a) {
  if (s->npred != S::MP || s->nvals != S::MV || s->naggs != S::MA) return false;
  for (int i = 0; i < S::MA; ++i) {
    if (kinds[i] != (int)((S::kKinds >> (4 * i)) & 15u)) return false;
    if (a.expr[i] != (int)((S::kExprs >> (4 * i)) & 15u)) return false;
    const int nargs = a.expr[i] == NUT_EX_COL ? 1 : a.expr[i] == NUT_EX_MUL_1M_1P ? 3 : 2;
    for (int j = 0; j < 3; ++j) {
      int want = (int)((S::kArgs >> (6 * i + 2 * j)) & 3u);
      if (kinds[i] != AK_COUNT && j < nargs && a.arg[i][j] != want) return false;
    }
  }
  for (int t = 0; t < S::MP; ++t)
    if (a.pred_type[t] != (int)((S::kPreds >> (4 * t + 3)) & 1u) || a.pred_op[t] != (int)((S::kPreds >> (4 * t)) & 7u))
      return false;
  for (int c = 0; c < S::MV; ++c)
    if (s->val_type[c] != NUT_T_F64) return false;
  return true;
}

int detect_shape(const nut_agg_spec *s, const int32_t *kinds, const AggArgs &a) {
  if (s->nkeys == 2 && shape_matches<ShapeQ1>(s, kinds, a)) return SHAPE_Q1;
  if (s->nkeys == 1 && shape_matches<ShapeSum>(s, kinds, a)) return SHAPE_SUM;
  if (s->nkeys == 1 && shape_matches<ShapeSumCount>(s, kinds, a)) return SHAPE_SUMCOUNT;
  if (s->nkeys == 1 && shape_matches<ShapeAll4>(s, kinds, a)) return SHAPE_ALL4;
  return SHAPE_GENERIC;
}

constexpr int kBdShared = 512;
constexpr int kBdPriv = 256;

// Compiled shapes assume 16-B aligned columns (vector loads); anything else runs the
// generic kernel, which decides the load width at run time.
KernelFn pick_kernel(int nk, bool priv, int shape, bool vec, int bd) {
  if (!vec) shape = SHAPE_GENERIC;
  if (priv) {
    if (shape == SHAPE_Q1)
      return bd == 128 ? agg_kernel<2, true, 128, ShapeQ1, 1>
           : bd == 192 ? agg_kernel<2, true, 192, ShapeQ1, 1> : agg_kernel<2, true, kBdPriv, ShapeQ1, 1>;
    if (shape == SHAPE_SUM) return agg_kernel<1, true, kBdPriv, ShapeSum, 1>;
    if (shape == SHAPE_ALL4) return agg_kernel<1, true, kBdPriv, ShapeAll4, 1>;
    return nk == 1 ? agg_kernel<1, true, kBdPriv, Generic, 0> : agg_kernel<2, true, kBdPriv, Generic, 0>;
  }
  if (shape == SHAPE_Q1) return agg_kernel<2, false, kBdShared, ShapeQ1, 1>;
  if (shape == SHAPE_SUM) return agg_kernel<1, false, kBdShared, ShapeSum, 1>;
  if (shape == SHAPE_SUMCOUNT) return agg_kernel<1, false, kBdShared, ShapeSumCount, 1>;
  if (shape == SHAPE_ALL4) return agg_kernel<1, false, kBdShared, ShapeAll4, 1>;
  return nk == 1 ? agg_kernel<1, false, kBdShared, Generic, 0> : agg_kernel<2, false, kBdShared, Generic, 0>;
}

size_t lds_bytes(uint32_t cap, int nk, int na, bool priv, int P, int bd) {
  if (cap == 0) return 0;
  size_t a, b, c, d, e;
  return lds_layout(cap, nk, na, priv, P, bd, &a, &b, &c, &d, &e);
}

// Partitioned aggregation (gpart.hpp) drives the same kernels in two extra modes.
struct LaunchExtra {
  bool spill = false;                      // stage rows passing WHERE (no tables)
  uint64_t *sp_cols[3 + NUT_MAX_VALS] = {};
  unsigned long long *sp_counts = nullptr; // [blocks] rows staged per block
  unsigned long long *sp_hist = nullptr;   // [256] level-0 histogram (zeroed)
  int32_t sp_map[NUT_MAX_AGGS] = {};
  uint64_t blocks = 0, region = 0;         // out (spill): grid and per-block staging region
  const uint64_t *seg_off = nullptr;       // one block per segment: [start, end) pairs, even starts
  const uint64_t *seg_end = nullptr;       //   or starts in seg_off, ends here (AggArgs::seg_end)
  const uint64_t *seg_cut = nullptr;       //   ... or at min(seg_end, seg_cut) (AggArgs::seg_cut)
  uint32_t nseg = 0;
  bool dense = false;                      // every segment a whole partition (AggArgs::dense)
  unsigned long long *dcount = nullptr;    // dense staging (AggArgs::dcount / dregion / dbase)
  uint64_t dregion = 0, dbase = 0;
  bool dry = false;       // compute the launch configuration only (nothing is launched)
  bool q1_fused = false;  // out (dry): the launch takes the compiled Q1 kernel
};

// The compiled Q1 kernel's launch shapes, threads x workgroups per CU.  All run 6-8 waves
// per CU; which one streams the six columns best differs between boards (the driver's box
// reached 0.929 of its copy floor at 192 x 2 where builder boxes reached 0.97-1.0), so the
// first large launch on a device times each (probe_priv_shape) and the device keeps the
// fastest for the process.
constexpr int kPrivShapes[3][2] = {{192, 2}, {128, 3}, {128, 4}};
struct PrivShape {
  int shape = -1;  // index into kPrivShapes; -1: not probed (192 x 2)
  double ms[3] = {-1, -1, -1};
  double cost_ms = 0;  // wall time the probe added to the call that ran it (nut_ctx_priv_probe_cost)
};
static PrivShape g_priv_shape[64];
static std::mutex g_priv_mu;
static PrivShape priv_shape_of(int dev) {
  std::lock_guard<std::mutex> lk(g_priv_mu);
  return dev >= 0 && dev < 64 ? g_priv_shape[dev] : PrivShape{};
}

// the on-chip table of a launch: 4x the expected groups (load <= 1/4: a key almost always
// sits in its 4-slot home bucket) within the LDS budget; segment mode: NUT_OPT_GB_SEG_SLOTS x
// group_hint (already twice a partition's expected groups).  0: hot keys cannot fit on chip
constexpr size_t kAggLdsMax = 160 * 1024 - 2048;  // the kernel also holds static LDS (spill cursor, histogram)
uint32_t agg_lcap(nut_ctx *c, int nk, int na, uint64_t group_hint, bool seg) {
  // (32 slots = 8 buckets x 32 B = one pass over the 64 LDS banks: for <= 8 groups two
  // home buckets never conflict — distinct buckets hit distinct banks, equal ones broadcast)
  const uint64_t want = group_hint ? (uint64_t)c->opt[seg ? NUT_OPT_GB_SEG_SLOTS : NUT_OPT_AGG_SLOTS] * group_hint : 4096;
  uint32_t lcap = 32;
  while (lcap < want && lds_bytes(lcap * 2, nk, na, false, 0, kBdShared) <= kAggLdsMax) lcap *= 2;
  return group_hint > 8ull * lcap ? 0 : lcap;
}

// launch the streaming aggregation of spec's rows into g's table.  `kinds` are the
// per-row update kinds (COUNT partials are merged as integer sums).
nut_status launch_agg(nut_groups *g, const nut_agg_spec *s, uint64_t group_hint, const int32_t *kinds,
                      LaunchExtra *ex = nullptr) {
  g->ctl_valid = false;  // this launch writes the table
  nut_ctx *c = g->ctx;
  if (s->n == 0) return NUT_OK;
  AggArgs a;
  memset(&a, 0, sizeof(a));
  a.n = s->n;
  // nkeys == 0 (global aggregate) runs the one-key kernels with every key = 0
  a.nokey = s->nkeys == 0 ? 1 : 0;
  // (a computed key — key_prog — is evaluated in the kernel; its column pointer is unused)
  a.keys[0] = (const uint64_t *)(s->nkeys && !s->key_prog[0].n ? s->keys[0] : nullptr);
  a.keys[1] = s->nkeys == 2 && !s->key_prog[1].n ? (const uint64_t *)s->keys[1] : a.keys[0];
  a.npred = s->npred;
  for (int t = 0; t < s->npred; ++t) {
    a.pred_col[t] = (const uint64_t *)s->pred_col[t];
    a.pred_type[t] = s->pred_type[t];
    a.pred_op[t] = s->pred_op[t];
    if (s->pred_type[t] == NUT_T_I64) a.pred_k[t] = (uint64_t)s->pred_i64[t];
    else memcpy(&a.pred_k[t], &s->pred_f64[t], 8);
    if (s->pred_op[t] >= NUT_IN) {
      a.pred_nset[t] = s->pred_nset[t];
      for (int i = 0; i < s->pred_nset[t]; ++i) a.pred_set[t][i] = (uint64_t)s->pred_set[t][i];
    }
  }
  a.nvals = s->nvals;
  for (int v = 0; v < s->nvals; ++v) a.val_col[v] = (const uint64_t *)s->val_col[v];
  if (s->prog_mode) {
    a.nvals = s->nprog_cols;
    for (int v = 0; v < s->nprog_cols; ++v) a.val_col[v] = (const uint64_t *)s->prog_col[v];
  }
  a.naggs = s->naggs;
  a.kinds = pack_kinds(kinds, s->naggs);
  for (int i = 0; i < s->naggs; ++i) {
    a.expr[i] = s->agg_op[i] == NUT_AGG_COUNT ? NUT_EX_COL : s->agg_expr[i];
    for (int j = 0; j < 3; ++j) a.arg[i][j] = s->agg_op[i] == NUT_AGG_COUNT ? 0 : s->agg_arg[i][j];
  }
  auto misaligned = [](const void *ptr) { return ptr && ((uintptr_t)ptr & 15) != 0; };
  bool bad = misaligned(a.keys[0]) || misaligned(a.keys[1]);
  for (int t = 0; t < a.npred; ++t) bad |= misaligned(a.pred_col[t]);
  for (int v = 0; v < a.nvals; ++v) bad |= misaligned(a.val_col[v]);
  a.vec = bad ? 0 : 1;  // 8-B aligned columns (e.g. slices) take two 8-B loads per pair

  const size_t lds_max = kAggLdsMax;
  const int na = s->naggs;
  uint32_t lcap = agg_lcap(c, g->nk, na, group_hint, ex && ex->seg_off);
  if (ex && ex->spill) {
    lcap = 0;
    a.sp_counts = ex->sp_counts;
    a.sp_hist = ex->sp_hist;
    for (int i = 0; i < 3 + NUT_MAX_VALS; ++i) a.sp_cols[i] = ex->sp_cols[i];
    for (int i = 0; i < NUT_MAX_AGGS; ++i) a.sp_map[i] = ex->sp_map[i];
  }
  // private accumulators when every expected group fits P per thread, 2 blocks per CU
  int P = 0;
  if (lcap && group_hint && group_hint <= (uint64_t)kPrivMax && na > 0 && !(ex && ex->seg_off)) {
    P = (int)group_hint;
    if (lds_bytes(lcap, g->nk, na, true, P, kBdPriv) > lds_max / 2) P = 0;
  }
  const bool priv = P > 0;
  const int shape = detect_shape(s, kinds, a);
  // private-accumulator kernels built for 128 / 192 / 256 threads: the compiled Q1 shape
  // and every run-time-compiled (expression-mode) kernel
  const bool q1_tuned = priv && ((shape == SHAPE_Q1 && !s->prog_mode && a.vec) || s->prog_mode);
  // the Q1 kernel runs 6 waves per CU (2 x 192 threads): 8 waves issue too many
  // concurrent six-column streams (7.85 vs 7.27 ms at 1e9 rows, same box), 4 leave its
  // fold's latency exposed (8.7 ms) — NUT_OPT_PRIV_BD / _BLOCKS override for sweeps.  The
  // compiled (fused) Q1 kernel takes the shape its device's probe chose (kPrivShapes).
  const bool q1_fused = q1_tuned && !s->prog_mode;
  int pbd = 192, pblocks = 2;
  if (q1_fused) {
    const int k = c->priv_probe >= 0 ? c->priv_probe : priv_shape_of(c->device).shape;
    if (k >= 0) pbd = kPrivShapes[k][0], pblocks = kPrivShapes[k][1];
  }
  if (ex && ex->dry) {
    ex->q1_fused = q1_fused;
    return NUT_OK;
  }
  const int bd = !priv ? kBdShared : !q1_tuned ? kBdPriv : c->opt[NUT_OPT_PRIV_BD] ? (int)c->opt[NUT_OPT_PRIV_BD] : pbd;
  a.lds_cap = lcap;
  a.lds_limit = lcap - lcap / 4;
  a.lds_log2 = lcap ? ilog2(lcap) : 0;
  a.priv = P;
  a.gt = g->dev_gt;
  const size_t lb = lds_bytes(lcap, g->nk, na, priv, P, bd);
  int blocks_per_cu = lb ? (int)std::max<size_t>(1, std::min<size_t>(bd == 512 ? 4 : 8, lds_max / lb)) : 4;
  if (q1_tuned)
    blocks_per_cu = std::min<int>(blocks_per_cu, c->opt[NUT_OPT_PRIV_BLOCKS] ? (int)c->opt[NUT_OPT_PRIV_BLOCKS]
                                                 : q1_fused ? pblocks : 2);
  if (!priv && c->opt[NUT_OPT_AGG_BLOCKS]) blocks_per_cu = std::min<int>(blocks_per_cu, (int)c->opt[NUT_OPT_AGG_BLOCKS]);
  uint64_t pairs = (s->n + 1) / 2;
  uint64_t blocks = std::min<uint64_t>((uint64_t)c->num_cus * blocks_per_cu, (pairs + bd - 1) / bd);
  if (blocks == 0) blocks = 1;
  if (ex && ex->seg_off) {  // one block per segment (segments start at even rows)
    a.seg_off = ex->seg_off;
    a.seg_end = ex->seg_end;
    a.seg_cut = ex->seg_cut;
    a.dense = ex->dense && g->nk == 1 ? 1 : 0;
    blocks = ex->nseg;
    if (ex->dcount) {  // dense staging: every region must hold a full block table
      if (!a.dense || !lcap || ex->dregion < (uint64_t)lcap + 1)
        return fail(NUT_ERR_INVALID_ARG, "launch_agg: dense staging region smaller than the block table");
      a.dcount = ex->dcount;
      a.dregion = ex->dregion;
      a.dbase = ex->dbase;
    }
  }
  if (ex && ex->spill) {  // block b stages at most the rows it visits: 2 per pair of its lanes
    a.sp_region = 2ull * bd * ((pairs + blocks * bd - 1) / (blocks * bd));
    ex->blocks = blocks;
    ex->region = a.sp_region;
  }
  if (s->prog_mode) {
    // expression mode: the query's own kernel (jit.cpp), compiled once per shape
    JitShape js;
    nut_status st = jit_shape(s, kinds, js);
    if (st) return st;
    if (js.consts.size() > (size_t)kMaxConst)
      return fail(NUT_ERR_UNSUPPORTED, "nut_groupby: more than 64 distinct expression constants");
    for (size_t i = 0; i < js.consts.size(); ++i) a.kc[i] = js.consts[i];
    hipFunction_t fn;
    st = jit_kernel(jit_unit(js.src, g->nk, priv, bd, sizeof(AggArgs)), true, &fn);
    if (st) return st;
    size_t asz = sizeof(a);
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz, HIP_LAUNCH_PARAM_END};
    c->timer.begin(c->stream, NUT_KERNEL_AGGREGATE);
    hipError_t e = hipModuleLaunchKernel(fn, (unsigned)blocks, 1, 1, (unsigned)bd, 1, 1, (unsigned)lb, c->stream,
                                         nullptr, cfg);
    c->timer.end(c->stream);
    if (e != hipSuccess) return hip_fail(e, "hipModuleLaunchKernel (expression kernel)");
    return NUT_OK;
  }
  KernelFn fn = pick_kernel(g->nk, priv, shape, a.vec != 0, bd);
  NUT_HIP(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
  c->timer.begin(c->stream, NUT_KERNEL_AGGREGATE);
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(bd), lb, c->stream, a);
  c->timer.end(c->stream);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

uint64_t table_cap_for(uint64_t groups) {
  uint64_t cap = 1024;
  while (cap < 2 * groups) cap *= 2;
  return cap;
}

// grow the table (rehash existing groups) so that `extra` more groups fit
nut_status ensure_room(nut_groups *g, uint64_t extra) {
  uint32_t ctl[4];
  nut_status st = read_ctl(g, ctl);
  if (st) return st;
  uint64_t need = (uint64_t)ctl[0] + extra + 1;
  // sharded counters (large tables) overflow per shard: keep 1/8 of headroom for variance
  const uint64_t slack = g->gt.nsh_log2 ? need / 8 : 0;
  if (!g->dense && need + slack <= g->gt.limit && (g->nk == 1 || (uint64_t)ctl[3] + extra + slack <= g->gt.arena_cap))
    return NUT_OK;
  nut_groups fresh;
  fresh.ctx = g->ctx;
  fresh.nk = g->nk;
  fresh.naggs = g->naggs;
  memcpy(fresh.kinds, g->kinds, sizeof(g->kinds));
  st = alloc_table(&fresh, table_cap_for(need));
  if (st) return st;
  nut_ctx *c = g->ctx;
  uint64_t stride = g->gt.cap + 1;
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)c->num_cus * 8);
  hipLaunchKernelGGL(rehash_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, (const GTable *)g->dev_gt,
                     (const GTable *)fresh.dev_gt, g->nk);
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipStreamSynchronize(c->stream));
  (void)hipFree(g->mem);
  g->mem = fresh.mem;
  g->mem_bytes = fresh.mem_bytes;
  g->gt = fresh.gt;
  g->dev_gt = fresh.dev_gt;
  g->ctl_valid = false;
  g->dev_cursors = fresh.dev_cursors;
  g->dev_segbase = fresh.dev_segbase;
  g->dense = false;
  fresh.mem = nullptr;
  return NUT_OK;
}

// ---------------------------------------------------------------- partitioned aggregation
// (gpart.hpp).  Used when the expected groups exceed what the on-chip tables hold.
// nut_ctx_set_option NUT_OPT_GB_PARTITION / NUT_OPT_GB_LEVELS force the path and its
// levels (tests drive them at small sizes).
constexpr uint64_t kGpMinGroups = 1ull << 16;

// upload host vectors into a fresh region of ctx->gp_meta (grown after a sync)
struct GpMeta {
  nut_ctx *c;
  size_t off = 0;
  std::vector<std::vector<char>> keep;
  static size_t al(size_t x) { return (x + 255) & ~size_t(255); }
  nut_status begin(size_t total) {
    off = 0;
    total += 16 * 256;  // (up() adds a byte to every upload: one extra 256-B unit each, <= 16 per call)
    if (total > c->gp_meta.bytes) {
      NUT_HIP(hipStreamSynchronize(c->stream));
      nut_status s = c->gp_meta.reserve(total);
      if (s) return s;
    }
    return NUT_OK;
  }
  void *alloc(size_t b) {
    void *p = (char *)c->gp_meta.ptr + off;
    off += al(b);
    return p;
  }
  template <class T>
  nut_status up(const std::vector<T> &v, T **d) {
    *d = (T *)alloc(v.size() * sizeof(T) + 1);
    if (v.empty()) return NUT_OK;
    keep.emplace_back((const char *)v.data(), (const char *)(v.data() + v.size()));
    NUT_HIP(hipMemcpyAsync(*d, keep.back().data(), v.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return NUT_OK;
  }
};

uint32_t gp_tiles(std::vector<GpSeg> &segs, uint32_t tile, std::vector<uint32_t> &ts) {
  ts.clear();
  for (uint32_t i = 0; i < segs.size(); ++i) {
    segs[i].tile0 = (uint32_t)ts.size();
    ts.insert(ts.end(), (segs[i].count + tile - 1) / tile, i);
  }
  return (uint32_t)ts.size();
}

// the capped scatter launch (no histogram; see gp_level): hash digits, or range digits of
// one key (rg: GpRange, t >= 0 ... the ordered group-by)
void gp_capped_launch(nut_ctx *c, const GpArrays &ar, const GpSeg *dseg, const uint32_t *dts, uint32_t nst, int shift,
                      unsigned long long *dcur, uint64_t kx, uint64_t ovf, unsigned long long *dflag, int bits,
                      bool two_keys, const GpRange *rg, unsigned long long *acur = nullptr, uint64_t acap = 0,
                      unsigned long long *acut = nullptr, int gather = 0, int threads = 1024, int spare_cus = 0) {
  if (!nst) return;
  // persistent workgroups, one per CU — less `spare_cus`, CUs left to run other streams'
  // kernels beside this launch (the ordered path's aggregation of the previous chunk)
  const unsigned grid = std::min<unsigned>(nst, (unsigned)std::max(1, c->num_cus - spare_cus));
  using SK = void (*)(GpArrays, const GpSeg *, const uint32_t *, uint32_t, int, int, unsigned long long *, uint64_t,
                      uint64_t, unsigned long long *, GpRange, unsigned long long *, uint64_t, unsigned long long *);
  static const SK kern[3][3] = {
      {gp_scatter_kernel<1, 1024, 1, 6>, gp_scatter_kernel<1, 1024, 1, 7>, gp_scatter_kernel<1, 1024, 1, 8>},
      {gp_scatter_kernel<2, 1024, 1, 6>, gp_scatter_kernel<2, 1024, 1, 7>, gp_scatter_kernel<2, 1024, 1, 8>},
      {gp_scatter_kernel<1, 1024, 1, 6, true>, gp_scatter_kernel<1, 1024, 1, 7, true>,
       gp_scatter_kernel<1, 1024, 1, 8, true>}};
  // range digits at 512 threads (8 Ki-record tiles, ~75 KB of LDS): the ordered path's level
  // 1 can then share each CU with an aggregation workgroup (NUT_OPT_GB_L1_THREADS)
  static const SK kern512[3] = {gp_scatter_kernel<1, 512, 1, 6, true>, gp_scatter_kernel<1, 512, 1, 7, true>,
                                gp_scatter_kernel<1, 512, 1, 8, true>};
  const int kv = rg ? 2 : two_keys ? 1 : 0;
  const bool narrow = rg && threads == 512;
  hipLaunchKernelGGL(narrow ? kern512[bits - 6] : kern[kv][bits - 6], dim3(grid), dim3(narrow ? 512 : 1024), 0,
                     c->stream, ar, dseg, dts, nst, shift, gather, dcur, kx, ovf, dflag, rg ? *rg : GpRange{}, acur,
                     acap, acut);
}

// one partition level: histogram + scatter of every segment; returns the 256 counts per
// segment in `hist` (gather mode: one histogram for all segments; `have_hist`: the caller
// already holds it — the spill pass counts level 0)
// `parts` (if not null): the output is laid out as 256 partitions per input segment, each
// starting at an even row (16-B aligned for the aggregation's vector loads); their
// [start, end) pairs are appended to *parts
nut_status gp_level(nut_ctx *c, GpMeta &mm, std::vector<GpSeg> &segs, int shift, const uint64_t *const *src,
                    uint64_t *const *dst, int narr, bool gather, bool have_hist, std::vector<uint64_t> &hist,
                    std::vector<uint64_t> *parts = nullptr, uint64_t kx = 0, uint64_t ovf = 0, int bits = 8,
                    const GpRange *rg = nullptr, unsigned long long *acur = nullptr, uint64_t acap = 0) {
  hipStream_t st = c->stream;
  std::vector<uint32_t> ts;
  nut_status s;
  GpSeg *dseg;
  uint32_t *dts;
  const size_t nh = gather ? 1 : segs.size();  // gather: every segment into one compact range
  if (ovf) {
    // capped layout (no histogram pass): digit d of segment i owns rows [obase + d * ocap,
    // obase + (d + 1) * ocap) of dst (both even: 16-B aligned partitions), set by the
    // caller; the counts are the cursors read back after the scatter; rows [ovf, ovf +
    // 16 Ki) of every dst array must exist (overflowing runs land there).  NUT_ERR_CAPACITY
    // (no message) if a digit outgrew its rows: nothing is usable, partition again with a
    // histogram.  With an overflow arena (acur) an overflowing run goes there instead and
    // its digit's rows end at the first such run (see gp_scatter_kernel).
    // (bits: the digit width of this level, 6..8).  Gather: every segment scatters into
    // segment 0's regions (the segments must name the same obase / ocap).
    if (have_hist || !parts || bits < 6 || bits > 8)
      return fail(NUT_ERR_INVALID_ARG, "gp_level: capped layout needs parts");
    const int nb = 1 << bits;
    const size_t nc = nh * nb;
    std::vector<uint64_t> cur(nc + 1, 0);  // + the overflow flag
    for (size_t i = 0; i < segs.size(); ++i) {
      if ((segs[i].obase | segs[i].ocap) & 1) return fail(NUT_ERR_INVALID_ARG, "gp_level: odd capped region");
      if (gather && (segs[i].obase != segs[0].obase || segs[i].ocap != segs[0].ocap))
        return fail(NUT_ERR_INVALID_ARG, "gp_level: gathered capped segments name different regions");
      if (i < nh)
        for (int d = 0; d < nb; ++d) cur[i * nb + d] = segs[i].obase + (uint64_t)d * segs[i].ocap;
    }
    const uint32_t nst = gp_tiles(segs, 2 * GP_TILE, ts);
    s = mm.begin(GpMeta::al(segs.size() * sizeof(GpSeg)) + GpMeta::al(ts.size() * 4 + 1) + GpMeta::al(cur.size() * 8) +
                 (acur ? GpMeta::al(nc * 8) : 0));
    if (s) return s;
    uint64_t *dcur;
    if ((s = mm.up(segs, &dseg)) || (s = mm.up(ts, &dts)) || (s = mm.up(cur, &dcur))) return s;
    unsigned long long *dcut = nullptr;  // first overflowing run per digit (none: ~0)
    if (acur) {
      dcut = (unsigned long long *)mm.alloc(nc * 8);
      NUT_HIP(hipMemsetAsync(dcut, 0xff, nc * 8, st));
    }
    GpArrays ar;
    for (int a = 0; a < GP_MAX_ARR; ++a) {
      ar.src[a] = src[a];
      ar.dst[a] = dst[a];
    }
    ar.narr = narr;
    unsigned long long *dflag = (unsigned long long *)dcur + nc;
    gp_capped_launch(c, ar, dseg, dts, nst, shift, (unsigned long long *)dcur, kx, ovf, dflag, bits, src[2] != nullptr,
                     rg, acur, acap, dcut, gather ? 1 : 0);
    NUT_HIP(hipGetLastError());
    std::vector<uint64_t> back(cur.size()), cut(dcut ? nc : 0);
    NUT_HIP(hipMemcpyAsync(back.data(), dcur, back.size() * 8, hipMemcpyDeviceToHost, st));
    if (dcut) NUT_HIP(hipMemcpyAsync(cut.data(), dcut, nc * 8, hipMemcpyDeviceToHost, st));
    NUT_HIP(hipStreamSynchronize(st));
    if (back[nc]) return NUT_ERR_CAPACITY;
    for (size_t i = 0; i < cut.size(); ++i) back[i] = std::min(back[i], cut[i]);
    hist.assign(nc, 0);
    for (size_t i = 0; i < nc; ++i) {
      hist[i] = back[i] - cur[i];
      if (hist[i]) {
        parts->push_back(cur[i]);
        parts->push_back(back[i]);
      }
    }
    return NUT_OK;
  }
  if (!have_hist) {
    const uint32_t nht = gp_tiles(segs, GP_HTILE, ts);
    const size_t hb = nh * GP_BINS * 8;
    s = mm.begin(GpMeta::al(segs.size() * sizeof(GpSeg)) + GpMeta::al(ts.size() * 4 + 1) + GpMeta::al(hb));
    if (s) return s;
    if ((s = mm.up(segs, &dseg)) || (s = mm.up(ts, &dts))) return s;
    unsigned long long *dh = (unsigned long long *)mm.alloc(hb);
    NUT_HIP(hipMemsetAsync(dh, 0, hb, st));
    if (nht) hipLaunchKernelGGL(gp_hist_kernel, dim3(nht), dim3(GP_HTHREADS), 0, st, src[1], src[2],
                                (const GpSeg *)dseg, (const uint32_t *)dts, shift, gather ? 1 : 0, dh, kx);
    NUT_HIP(hipGetLastError());
    hist.resize(nh * GP_BINS);
    NUT_HIP(hipMemcpyAsync(hist.data(), dh, hb, hipMemcpyDeviceToHost, st));
    NUT_HIP(hipStreamSynchronize(st));
  }
  std::vector<uint64_t> cur(hist.size());
  uint64_t arun = 0;  // aligned layout: one running offset over all (segment, digit)
  for (size_t i = 0; i < nh; ++i) {
    uint64_t run = gather ? 0 : segs[i].start;
    for (int d = 0; d < GP_BINS; ++d) {
      const uint64_t h = hist[i * GP_BINS + d];
      if (parts) {
        arun = (arun + 1) & ~1ull;
        cur[i * GP_BINS + d] = arun;
        if (h) {
          parts->push_back(arun);
          parts->push_back(arun + h);
        }
        arun += h;
      } else {
        cur[i * GP_BINS + d] = run;
        run += h;
      }
    }
  }
  // 1024-thread workgroups of 16K-record tiles (one per CU): 64 records per digit per tile;
  // measured 9.2 vs 10.1 ms for 512-thread 8K tiles at two per CU (G = 1e5, 1e9 rows)
  const uint32_t nst = gp_tiles(segs, 2 * GP_TILE, ts);
  s = mm.begin(GpMeta::al(segs.size() * sizeof(GpSeg)) + GpMeta::al(ts.size() * 4 + 1) + GpMeta::al(cur.size() * 8));
  if (s) return s;
  uint64_t *dcur;
  if ((s = mm.up(segs, &dseg)) || (s = mm.up(ts, &dts)) || (s = mm.up(cur, &dcur))) return s;
  GpArrays ar;
  for (int a = 0; a < GP_MAX_ARR; ++a) {
    ar.src[a] = src[a];
    ar.dst[a] = dst[a];
  }
  ar.narr = narr;
  if (nst) {
    const unsigned grid = std::min<unsigned>(nst, (unsigned)c->num_cus);
    if (src[2])
      hipLaunchKernelGGL((gp_scatter_kernel<2, 1024>), dim3(grid), dim3(1024), 0, st, ar, (const GpSeg *)dseg,
                         (const uint32_t *)dts, nst, shift, gather ? 1 : 0, (unsigned long long *)dcur, kx, 0,
                         (unsigned long long *)nullptr, GpRange{});
    else
      hipLaunchKernelGGL((gp_scatter_kernel<1, 1024>), dim3(grid), dim3(1024), 0, st, ar, (const GpSeg *)dseg,
                         (const uint32_t *)dts, nst, shift, gather ? 1 : 0, (unsigned long long *)dcur, kx, 0,
                         (unsigned long long *)nullptr, GpRange{});
  }
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

// per-partition aggregation of partitioned records (final level's `parts`) into g's table
nut_status gp_aggregate(nut_groups *g, GpMeta &mm, const std::vector<uint64_t> &parts, const nut_agg_spec &s2,
                        const int32_t *kinds2, uint64_t group_hint) {
  nut_ctx *c = g->ctx;
  hipStream_t st = c->stream;
  const uint32_t nparts = (uint32_t)(parts.size() / 2);
  if (nparts == 0) return NUT_OK;
  // split partitions into chunks (even boundaries) so that the grid fills the chip (chunks
  // of one partition merge the same keys: a handful of extra merges per group)
  const uint64_t wpc = (uint64_t)std::max<int64_t>(1, c->opt[NUT_OPT_GB_CHUNKS]);  // workgroups per CU (4: +0.12 ms at G = 1e5)
  const uint64_t k = std::max<uint64_t>(1, ((uint64_t)c->num_cus * wpc + nparts - 1) / nparts);
  std::vector<uint64_t> off;
  for (uint32_t p = 0; p < nparts; ++p) {
    const uint64_t a0 = parts[2 * p], a1 = parts[2 * p + 1];
    uint64_t prev = a0;
    for (uint64_t j = 1; j <= k; ++j) {
      const uint64_t cut = j == k ? a1 : std::max<uint64_t>(prev, (a0 + (a1 - a0) * j / k) & ~1ull);
      if (cut > prev) {
        off.push_back(prev);
        off.push_back(cut);
        prev = cut;
      }
    }
  }
  nut_status e = mm.begin(GpMeta::al(off.size() * 8));
  if (e) return e;
  uint64_t *doff;
  if ((e = mm.up(off, &doff))) return e;
  LaunchExtra sg;
  sg.seg_off = doff;
  sg.nseg = (uint32_t)(off.size() / 2);
  // one chunk per partition: its groups are final in its block, appended without hashing
  // (a partition with more groups than its block's table admits reruns hashed)
  sg.dense = k == 1 && g->nk == 1 && c->opt[NUT_OPT_GB_DENSE] != 0;
  const uint64_t per = std::max<uint64_t>(64, 2 * ((group_hint + nparts - 1) / nparts));
  uint32_t ctl[4];
  for (int attempt = 0;; ++attempt) {
    e = launch_agg(g, &s2, per, kinds2, &sg);
    if (!e) e = read_ctl(g, ctl);
    if (e) return e;
    if (ctl[1] & 4u) {  // dense: a block could not hold its partition — the hashed merge
      sg.dense = false;
      e = alloc_table(g, g->gt.cap);
      if (e) return e;
      continue;
    }
    g->dense = sg.dense;
    if (!(ctl[1] & 1u)) break;
    // more groups than the table admits: a larger table, then the same partitions again
    if (g->gt.cap >= (1ull << 34) || attempt > 12) return fail(NUT_ERR_OOM, "nut_groupby: group table too large");
    e = alloc_table(g, g->gt.cap * 4);
    if (e) return e;
  }
  NUT_HIP(hipStreamSynchronize(st));  // the host tables in mm.keep outlive their copies
  return NUT_OK;
}

// Spill-free partitioned aggregation (no WHERE, plain-column arguments): the key and value
// columns are partitioned by the key hash straight from the caller's columns.
nut_status groupby_partitioned_direct(nut_groups *g, const nut_agg_spec *s, uint64_t group_hint) {
  nut_ctx *c = g->ctx;
  hipStream_t st = c->stream;
  const int nk = g->nk, na = g->naggs;
  const uint64_t n = s->n;
  // value columns the aggregates read, each partitioned once
  int vmap[NUT_MAX_VALS];
  int nv = 0;
  for (int j = 0; j < NUT_MAX_VALS; ++j) vmap[j] = -1;
  for (int a = 0; a < na; ++a)
    if (s->agg_op[a] != NUT_AGG_COUNT && vmap[s->agg_arg[a][0]] < 0) vmap[s->agg_arg[a][0]] = nv++;
  const int narr = 3 + nv;
  const uint64_t rows = (n + 2 * 65536 + 64 + 31) & ~31ull;  // + one alignment gap per partition
  const int nstore = narr - 1 - (nk == 1 ? 1 : 0);
  const int levels = c->opt[NUT_OPT_GB_LEVELS] ? (int)c->opt[NUT_OPT_GB_LEVELS] : group_hint > 256ull * 1024 ? 2 : 1;
  const bool opt = c->opt[NUT_OPT_GB_OPTIMISTIC] != 0;
  c->gb_path = NUT_GB_PARTITIONED_DIRECT;
  c->gb_levels = (uint32_t)levels;
  c->gb_optimistic = 0;
  // Capped level 1 (bits1-bit digits; 6 by default — 64-bin runs are 4x longer than 256-bin
  // ones and 16384 partitions of ~610 groups aggregate faster than 65536 of ~150: same-box
  // A/B at G = 1e7, 1e9 rows, 19.9 vs 22.7 ms kernels): a level-1 partition's rows are about (rows per key) x
  // Poisson(lambda) with lambda = G / (256 << bits1) keys per partition, so a sub-digit owns
  // its even share times 1 + 6 / sqrt(lambda) (six standard deviations), + 64 rows —
  // offered from lambda >= 100 (slack <= 1.6x); below, level 1 takes the histogram layout.
  // level 0's digit: 7 bits for one level up to 150 K groups (128 partitions of <= ~1200
  // groups still fit a workgroup's 2048-slot table; the runs are twice as long: G = 1e5
  // 9.98 vs 10.56 ms kernels, same box), else 8 (two levels: G = 1e7 18.4 vs 18.6 ms)
  const int bits0 = c->opt[NUT_OPT_GB_L0_BITS] >= 6 ? (int)c->opt[NUT_OPT_GB_L0_BITS]
                    : levels == 1 && group_hint <= 150000 ? 7 : 8;
  const int bits1 = (int)c->opt[NUT_OPT_GB_L1_BITS];
  const double lam = (double)group_hint / ((double)(1 << bits0) * (1 << bits1));
  const double slack1 = levels == 2 && opt && lam >= 100 ? 1.0 + 6.0 / sqrt(lam) : 0.0;
  // A, B: the histogram layout (level 0 -> A -> level 1 -> B, or level 0 -> B); O: the
  // optimistic level 0 (2 x rows per array over A + B); B2: two levels' final arrays after O,
  // b2rows each
  const uint64_t b2rows = slack1 > 0 ? ((uint64_t)ceil(n * slack1) + (66ull << (bits0 + bits1)) + 2 * GP_TILE + 64 + 31) & ~31ull
                                     : rows;
  const bool two_opt = levels == 2 && opt;
  nut_status e = c->gp_data.reserve((2 * (size_t)nstore * rows + (two_opt ? (size_t)nstore * b2rows : 0)) * 8 + 256);
  if (e) return e;
  uint64_t *A[GP_MAX_ARR] = {}, *B[GP_MAX_ARR] = {}, *O[GP_MAX_ARR] = {}, *B2[GP_MAX_ARR] = {};
  for (int i = 1, k = 0; i < narr; ++i) {
    if (i == 2 && nk == 1) continue;
    A[i] = (uint64_t *)c->gp_data.ptr + (size_t)k * rows;
    B[i] = (uint64_t *)c->gp_data.ptr + (size_t)(nstore + k) * rows;
    O[i] = (uint64_t *)c->gp_data.ptr + (size_t)k * 2 * rows;
    B2[i] = (uint64_t *)c->gp_data.ptr + 2 * (size_t)nstore * rows + (size_t)k * b2rows;
    ++k;
  }
  // optimistic level 0 (bits0-bit digits): no histogram pass; a digit owns twice its even
  // share of rows (the rows after the partitions take overflowing runs: at least one tile),
  // so only a key hash skewed that far falls back to the histogram layout (8-bit digits)
  const uint64_t ocap = ((2 * rows - 2 * GP_TILE) >> bits0) & ~1ull;
  const uint64_t *src[GP_MAX_ARR] = {};
  src[1] = (const uint64_t *)s->keys[0];
  src[2] = nk == 2 ? (const uint64_t *)s->keys[1] : nullptr;
  for (int j = 0; j < NUT_MAX_VALS; ++j)
    if (vmap[j] >= 0) src[3 + vmap[j]] = (const uint64_t *)s->val_col[j];
  GpMeta mm{c};
  c->timer.begin(st, NUT_KERNEL_AGGREGATE);
  std::vector<GpSeg> segs{GpSeg{0, n, 0, 0}};
  segs[0].ocap = ocap;
  std::vector<uint64_t> hist, parts;
  uint64_t **fin = B;
  int shift1 = 48;  // level 1's digit: below level 0's
  if (levels == 1) {
    e = opt ? gp_level(c, mm, segs, 64 - bits0, src, O, narr, false, false, hist, &parts, 0, ocap << bits0, bits0)
            : NUT_ERR_CAPACITY;
    if (!e) {
      fin = O;
      c->gb_optimistic = 1;
    }
    if (e == NUT_ERR_CAPACITY) {
      hist.clear();
      parts.clear();
      e = gp_level(c, mm, segs, 56, src, B, narr, false, false, hist, &parts);
    }
    if (e) return e;
  } else {
    std::vector<GpSeg> s2;
    std::vector<uint64_t> p0;
    uint64_t **mid = A;
    uint64_t ovf1 = 0;  // capped level 1: its overflow rows (0: histogram layout)
    e = opt ? gp_level(c, mm, segs, 64 - bits0, src, O, narr, false, false, hist, &p0, 0, ocap << bits0, bits0)
            : NUT_ERR_CAPACITY;
    if (!e) {
      shift1 = 64 - bits0 - bits1;
      // level 1 without a histogram pass either (slack1 above; a skewed next hash byte
      // overflows and takes the histogram layout)
      for (size_t i = 0; i < p0.size(); i += 2) {
        GpSeg sg{p0[i], p0[i + 1] - p0[i], 0, 0};
        sg.obase = ovf1;
        sg.ocap = ((uint64_t)ceil((double)sg.count / (1 << bits1) * slack1) + 64 + 1) & ~1ull;
        ovf1 += (uint64_t)sg.ocap << bits1;
        s2.push_back(sg);
      }
      if (slack1 <= 0 || ovf1 + 2 * GP_TILE > b2rows) ovf1 = 0;
      mid = O;
      fin = B2;
      c->gb_optimistic = 1;
    } else if (e == NUT_ERR_CAPACITY) {
      hist.clear();
      e = gp_level(c, mm, segs, 56, src, A, narr, false, false, hist);
      if (e) return e;
      uint64_t run = 0;
      for (int d = 0; d < GP_BINS; ++d) {
        if (hist[d]) s2.push_back(GpSeg{run, hist[d], 0, 0});
        run += hist[d];
      }
    } else {
      return e;
    }
    std::vector<uint64_t> h2;
    e = ovf1 ? gp_level(c, mm, s2, shift1, mid, fin, narr, false, false, h2, &parts, 0, ovf1, bits1)
             : NUT_ERR_CAPACITY;
    if (!e) c->gb_optimistic = 2;
    if (e == NUT_ERR_CAPACITY) {
      h2.clear();
      parts.clear();
      e = gp_level(c, mm, s2, 48, mid, fin, narr, false, false, h2, &parts);
    }
    if (e) return e;
  }
  c->timer.end(st);
  nut_agg_spec s2;
  memset(&s2, 0, sizeof(s2));
  s2.n = n;  // (segment mode reads only the listed ranges)
  s2.nkeys = nk;
  s2.keys[0] = (const int64_t *)fin[1];
  s2.keys[1] = nk == 2 ? (const int64_t *)fin[2] : nullptr;
  s2.nvals = nv;
  s2.naggs = na;
  for (int j = 0; j < NUT_MAX_VALS; ++j)
    if (vmap[j] >= 0) {
      s2.val_col[vmap[j]] = fin[3 + vmap[j]];
      s2.val_type[vmap[j]] = s->val_type[j];
    }
  for (int a = 0; a < na; ++a) {
    s2.agg_op[a] = s->agg_op[a];
    s2.agg_expr[a] = NUT_EX_COL;
    if (s->agg_op[a] != NUT_AGG_COUNT) s2.agg_arg[a][0] = vmap[s->agg_arg[a][0]];
  }
  return gp_aggregate(g, mm, parts, s2, g->kinds, group_hint);
}

// ------------------------------------------------------------ ordered group-by (to host)
// A table for dense staging (AggArgs::dcount): `slots` slots and their aggregate words, no
// hashing, nothing initialised but the control words.
nut_status alloc_stage(nut_groups *g, uint64_t slots) {
  g->ctl_valid = false;
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  const size_t o_slot = carve(slots * 8), o_agg = carve(slots * 8 * (size_t)std::max(g->naggs, 1));
  const size_t o_ctl = carve(64), o_sh = carve(16 * 4), o_gt = carve(sizeof(GTable)), o_cur = carve(64 * 8),
               o_seg = carve(128 * 8);
  if (!(g->mem && g->mem_bytes >= off)) {
    if (g->mem) (void)hipFree(g->mem);
    g->mem = nullptr;
    nut_status ps = pool_take(g->ctx, off, &g->mem, &g->mem_bytes);
    if (ps) return ps;
  }
  char *b = (char *)g->mem;
  GTable &t = g->gt;
  memset(&t, 0, sizeof(t));
  t.slot = (uint64_t *)(b + o_slot);
  t.agg = (uint64_t *)(b + o_agg);
  t.ctl = (uint32_t *)(b + o_ctl);
  t.shard = (uint32_t *)(b + o_sh);
  t.cap = slots - 1;  // (stride = slots)
  t.log2cap = ilog2(slots);
  t.naggs = g->naggs;
  t.kinds = pack_kinds(g->kinds, g->naggs);
  g->dev_gt = (GTable *)(b + o_gt);
  g->dev_cursors = (unsigned long long *)(b + o_cur);
  g->dev_segbase = (uint64_t *)(b + o_seg);
  NUT_HIP(hipMemsetAsync(t.ctl, 0, 64, g->ctx->stream));
  NUT_HIP(hipMemcpyAsync(g->dev_gt, &g->gt, sizeof(GTable), hipMemcpyHostToDevice, g->ctx->stream));
  return NUT_OK;
}

bool host_pinned_ptr(const void *p) {
  hipPointerAttribute_t pa;
  const bool ok = p && hipPointerGetAttributes(&pa, p) == hipSuccess && pa.type == hipMemoryTypeHost;
  (void)hipGetLastError();  // pageable memory reports an error here
  return ok;
}

// The ordered group-by of config 3's shape at large G (one key, plain columns, no WHERE),
// straight into page-locked host arrays: the two capped partition levels take RANGE digits
// (GpRange over a sampled key range, 2^14 cells), so the 16384 final partitions are in key
// order and every one is final in its workgroup; each workgroup stages its groups, a
// per-partition pass ranks them by key and writes them to the ordered result at a prefix
// offset.  Level 1, the aggregation and the ordering run in chunks of level-0 partitions,
// and each finished chunk crosses to the host on a second stream while the next one is
// computed (the 16 B/group result at 1e7 groups is ~4.7 ms of PCIe): no device sort, no
// placement, and most of the transfer hidden.  NUT_ERR_UNSUPPORTED: not this shape, or the
// keys' spread or a partition overflowed the capped layout — the caller takes the hashed
// path (the host arrays may hold partial output then; it rewrites them).

// fold_sorted_groups (fold.hpp): its kinds are the tables' AggKind values
static_assert(fold::kSumF64 == AK_SUM_F64 && fold::kMinF64 == AK_MIN_F64 && fold::kMaxF64 == AK_MAX_F64 &&
                  fold::kMinI64 == AK_MIN_I64 && fold::kMaxI64 == AK_MAX_I64,
              "fold.hpp kinds");
using fold::fold_sorted_groups;

nut_status groupby_ordered(nut_ctx *c, const nut_agg_spec *s, uint64_t group_hint, int64_t *keys_h, uint64_t *aggs_h,
                           uint64_t cap, uint64_t *n_out) {
  const uint64_t n = s->n;
  const int na = s->naggs;
  bool shape = s->nkeys == 1 && !s->prog_mode && s->npred == 0 && !s->key_prog[0].n && c->opt[NUT_OPT_GB_ORDERED] != 0 &&
               c->opt[NUT_OPT_GB_DIRECT] != 0 && c->opt[NUT_OPT_GB_OPTIMISTIC] != 0 && c->opt[NUT_OPT_GB_PARTITION] != 0 &&
               c->opt[NUT_OPT_GB_LEVELS] != 1 && c->opt[NUT_OPT_GB_DENSE] != 0 && na >= 1 && n >= (1ull << 24) &&
               n >= 4 * group_hint && host_pinned_ptr(keys_h) && host_pinned_ptr(aggs_h) && cap > 0;
  for (int a = 0; a < na && shape; ++a) shape = s->agg_op[a] == NUT_AGG_COUNT || s->agg_expr[a] == NUT_EX_COL;
  // the 2^14 range cells split into a level-0 and a level-1 digit (NUT_OPT_GB_L0_BITS 6..8;
  // default 7 + 7: level 0's runs twice as long as at 8 + 6 for level 1's half as long —
  // same-box A/B at G = 1e7, 1e9 rows, three rounds: step 21.63-21.81 ms vs 22.44-22.56
  // (8 + 6) and 22.48-22.56 (6 + 8), profiles/r04/groupby1e7/ab_l0bits.txt)
  const int bits0 = c->opt[NUT_OPT_GB_L0_BITS] >= 6 && c->opt[NUT_OPT_GB_L0_BITS] <= 8 ? (int)c->opt[NUT_OPT_GB_L0_BITS] : 7;
  const int bits1 = 14 - bits0;
  const double lam = (double)group_hint / (double)(1 << (bits0 + bits1));
  c->gb_overflow_rows = 0;
  c->gb_decline = 0;
  c->gb_heavy_keys = 0;
  c->gb_heavy_rows = 0;
  // every NUT_ERR_UNSUPPORTED names its reason (nut_ctx_groupby_overflow): the caller then
  // runs the hashed path, with the same result
  auto decline = [c](uint32_t why) {
    c->gb_decline = why;
    return NUT_ERR_UNSUPPORTED;
  };
  if (!shape || lam < 100 || ((uintptr_t)s->keys[0] & 15)) return decline(NUT_GB_DECLINE_SHAPE);
  hipStream_t st = c->stream;
  // ---- the key range from a strided sample (+ 1/1024 of the span on either side)
  constexpr uint32_t kSample = 65536;
  nut_status e = c->misc.reserve(kSample * 8);
  if (e) return e;
  hipLaunchKernelGGL(go_sample_kernel, dim3(64), dim3(256), 0, st, s->keys[0], n, kSample, (int64_t *)c->misc.ptr);
  NUT_HIP(hipGetLastError());
  std::vector<int64_t> smp(kSample);
  NUT_HIP(hipMemcpyAsync(smp.data(), c->misc.ptr, kSample * 8, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  const auto mm2 = std::minmax_element(smp.begin(), smp.end());
  uint64_t lo = (uint64_t)*mm2.first ^ 0x8000000000000000ull, hi = (uint64_t)*mm2.second ^ 0x8000000000000000ull;
  const uint64_t margin = (hi - lo) >> 10;
  lo = lo > margin ? lo - margin : 0;
  hi = hi < ~0ull - margin ? hi + margin : ~0ull;
  GpRange rg{};
  rg.lo = lo;
  rg.span = hi - lo;
  if (rg.span < (1ull << 16)) return decline(NUT_GB_DECLINE_SHAPE);  // (mul must fit 32 bits; tiny spans hash fine)
  rg.t = rg.span >> 32 ? 32 - __builtin_clzll(rg.span) : 0;
  rg.mul = (uint32_t)((1ull << 46) / ((rg.span >> rg.t) + 1));
  // the sample's keys counted in an open-addressing table (2x the sample): distinct keys
  // for the admission, repeated ones for the heavy-key split (a sort of the 64 Ki keys took
  // milliseconds of host time ahead of every call's first kernel)
  constexpr uint32_t kSlots = 2 * kSample;
  std::vector<int64_t> tk(kSlots);
  std::vector<uint32_t> tc(kSlots, 0);
  for (int64_t k : smp) {
    uint32_t q = (uint32_t)(mix64((uint64_t)k) >> 32) & (kSlots - 1);
    while (tc[q] && tk[q] != k) q = (q + 1) & (kSlots - 1);
    tk[q] = k;
    ++tc[q];
  }
  {  // admission: the sample's distinct keys spread over the level-0 partitions.  Keys
     // clustered inside the sampled range would overfill some partitions' tables (each
     // holds ~2x its share of groups) and send the call to the hashed path after all the
     // work; decline up front instead.  Repeated keys count once: a heavy key is rows,
     // not groups (the heavy-key split or the overflow arenas below take its rows).
    const uint32_t np0 = 1u << bits0, bound = 2 * kSample / np0 + 16;
    std::vector<uint32_t> distinct(np0, 0);
    for (uint32_t q = 0; q < kSlots; ++q)
      if (tc[q]) ++distinct[rg.cell((uint64_t)tk[q]) >> bits1];
    for (uint32_t p = 0; p < np0; ++p)
      if (distinct[p] > bound) return decline(NUT_GB_DECLINE_CLUSTERED);
  }
  // ---- partition buffers: level 0 capped over O (2 x rows per array), level 1 into B2
  nut_groups *g = new nut_groups();
  struct Free {
    nut_groups *g;
    ~Free() { nut_groups_free(g); }
  } free_g{g};
  g->ctx = c;
  g->nk = 1;
  g->naggs = na;
  for (int a = 0; a < na; ++a) g->kinds[a] = kind_of(s, a);
  int vmap[NUT_MAX_VALS];
  int nv = 0;
  for (int j = 0; j < NUT_MAX_VALS; ++j) vmap[j] = -1;
  for (int a = 0; a < na; ++a)
    if (s->agg_op[a] != NUT_AGG_COUNT && vmap[s->agg_arg[a][0]] < 0) vmap[s->agg_arg[a][0]] = nv++;
  const int narr = 3 + nv, nstore = narr - 2;
  const uint64_t rows = (n + 2 * 65536 + 64 + 31) & ~31ull;
  // ---- heavy keys (heavy.hpp): a key the sample saw >= 3 times (expected rows >= ~1/22000
  // of the rows, most of a level-1 partition's share; a key of twice that share is still
  // sampled < 3 times one time in ten) would overflow its partition.  When such keys
  // hold >= 5 % of the sample, the <= HK_MAX most frequent are aggregated in one streaming
  // pass and the other rows, compacted into B2, are what the levels partition.
  std::vector<int64_t> hkeys;
  std::vector<uint16_t> hslot;
  uint64_t hseed1 = 0, hseed2 = 0;
  if (c->opt[NUT_OPT_GB_HEAVY] != 0) {
    std::vector<std::pair<uint32_t, int64_t>> cand;  // (sample count, key)
    for (uint32_t q = 0; q < kSlots; ++q)
      if (tc[q] >= 3) cand.emplace_back(tc[q], tk[q]);
    std::sort(cand.begin(), cand.end(), [](const auto &x, const auto &y) {
      return x.first > y.first || (x.first == y.first && x.second < y.second);
    });
    const size_t hmax = std::min<size_t>(HK_MAX, HK_WORDS / na);
    if (cand.size() > hmax) cand.resize(hmax);
    uint64_t cover = 0;
    for (const auto &x : cand) cover += x.first;
    if (cover * 20 >= kSample) {
      for (const auto &x : cand) hkeys.push_back(x.second);
      std::sort(hkeys.begin(), hkeys.end());
      // the pass's lookup table: a cuckoo table (two slots per key) built here, so every
      // lookup is two reads; new seeds if a key finds no place (at load <= 1/4, rare)
      hslot.assign(HK_SLOTS, 0);
      bool placed = false;
      for (uint64_t attempt = 0; attempt < 8 && !placed; ++attempt) {
        hseed1 = mix64(0x9E3779B97F4A7C15ull + 2 * attempt);
        hseed2 = mix64(0x9E3779B97F4A7C15ull + 2 * attempt + 1);
        placed = hk_cuckoo(hkeys.data(), (uint32_t)hkeys.size(), hseed1, hseed2, hslot.data());
      }
      if (!placed) hkeys.clear();  // (the overflow arenas take them)
    }
  }
  // Exact layout (heavy keys split off): the data is skewed below the heavy keys too
  // (Zipf-like: keys of ~1/2 to 2 partition shares remain), so the heavy pass's kept rows are
  // counted per range cell (go_cell_hist_kernel, 8 B per kept row) and both levels' regions
  // are laid out from the counts — no overflow, no arenas, no arena group-by or host fold.
  // NUT_OPT_GB_HEAVY = 2 keeps the capped layout behind the heavy pass (A/B, tests).
  const bool exact = !hkeys.empty() && c->opt[NUT_OPT_GB_HEAVY] != 2;
  // capped level-1 regions: the even share x slack1 (six standard deviations of a Poisson
  // count of lambda keys per partition); behind the heavy pass 2.5 x (1e9-row Zipf G = 1e7:
  // 62 M arena rows at 1.24 x)
  const double slack1 = exact ? 1.0 : hkeys.empty() ? 1.0 + 6.0 / sqrt(lam) : 2.5;
  // B2: the level-1 regions (n x slack1 + per-region slack), then level 1's overflow arena
  // (n / 2 rows, n / 4 with the wider regions, none exact), then one tile of scratch for
  // runs an exhausted arena cannot take
  const uint64_t arena1 = ((exact ? 0 : hkeys.empty() ? n / 2 : n / 4) + 31) & ~31ull;
  const uint64_t b2rows =
      ((uint64_t)ceil(n * slack1) + (66ull << (bits0 + bits1)) + arena1 + 2 * GP_TILE + 64 + 31) & ~31ull;
  // (no growth margin; buffers that do not fit send the call to the hashed path, which
  // needs less)
  e = c->gp_data.reserve((2 * (size_t)nstore * rows + (size_t)nstore * b2rows) * 8 + 256, false);
  if (e) {
    (void)hipGetLastError();
    return decline(NUT_GB_DECLINE_CAPACITY);
  }
  uint64_t *O[GP_MAX_ARR] = {}, *B2[GP_MAX_ARR] = {};
  for (int i = 1, k = 0; i < narr; ++i) {
    if (i == 2) continue;
    O[i] = (uint64_t *)c->gp_data.ptr + (size_t)k * 2 * rows;
    B2[i] = (uint64_t *)c->gp_data.ptr + 2 * (size_t)nstore * rows + (size_t)k * b2rows;
    ++k;
  }
  const uint64_t *src[GP_MAX_ARR] = {};
  src[1] = (const uint64_t *)s->keys[0];
  for (int j = 0; j < NUT_MAX_VALS; ++j)
    if (vmap[j] >= 0) src[3 + vmap[j]] = (const uint64_t *)s->val_col[j];
  GpMeta mm{c};
  c->gb_path = NUT_GB_PARTITIONED_ORDERED;
  c->gb_levels = 2;
  c->gb_optimistic = 2;
  // overflow arenas (a run past its capped region keeps its rows there, gpart.hpp), one
  // cursor per level: [0] level 0's (in O), [1] level 1's (in B2)
  unsigned long long *darena = nullptr;
  NUT_HIP(hipMallocAsync((void **)&darena, 16, st));
  struct FreeArena {
    unsigned long long *p;
    hipStream_t s;
    ~FreeArena() { (void)hipFreeAsync(p, s); }
  } free_arena{darena, st};
  NUT_HIP(hipMemsetAsync(darena, 0, 16, st));
  uint64_t n0 = n;  // the rows the partition levels read
  std::vector<uint64_t> hcount;  // heavy pass: the rows each workgroup kept, at hchunk-row strides of B2
  uint64_t hchunk = 0;
  unsigned long long *dheavy = nullptr;
  struct FreeHeavy {
    unsigned long long *p = nullptr;
    hipStream_t s;
    ~FreeHeavy() {
      if (p) (void)hipFreeAsync(p, s);
    }
  } free_heavy{nullptr, st};
  const uint32_t nh = (uint32_t)hkeys.size();
  std::vector<uint64_t> cells;  // exact: kept rows per range cell
  if (nh) {
    using HK = void (*)(HkArgs);
    static const HK hkern[NUT_MAX_VALS + 1] = {hk_split_kernel<0>, hk_split_kernel<1>, hk_split_kernel<2>,
                                               hk_split_kernel<3>, hk_split_kernel<4>};
    static_assert(NUT_MAX_VALS == 4, "one heavy-pass kernel per value-array count");
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hkern[nv], HK_THREADS, 0) != hipSuccess || per_cu < 1)
      per_cu = 1;
    const uint64_t ntiles = (n + HK_TILE - 1) / HK_TILE;
    const uint64_t hgrid = std::min<uint64_t>(ntiles, (uint64_t)c->num_cus * per_cu);
    const uint64_t chunk = (ntiles + hgrid - 1) / hgrid;
    if (chunk * HK_TILE * 8 >= (1ull << 32)) return decline(NUT_GB_DECLINE_CAPACITY);  // (a chunk's buffer resource)
    // [keys (h), aggregates (h x na), kept rows per workgroup (hgrid), cuckoo slots, exact:
    // kept rows per range cell]
    const size_t slot0 = nh + (size_t)nh * na + hgrid, cell0 = slot0 + HK_SLOTS / 4;
    std::vector<uint64_t> init(cell0 + (exact ? GO_CELLS : 0), 0);
    memcpy(&init[0], hkeys.data(), (size_t)nh * 8);
    memcpy(&init[slot0], hslot.data(), HK_SLOTS * 2);
    for (uint32_t j = 0; j < nh; ++j)
      for (int a = 0; a < na; ++a) init[nh + (size_t)j * na + a] = agg_init(g->kinds[a]);
    NUT_HIP(hipMallocAsync((void **)&dheavy, init.size() * 8, st));
    free_heavy.p = dheavy;
    NUT_HIP(hipMemcpyAsync(dheavy, init.data(), init.size() * 8, hipMemcpyHostToDevice, st));
    HkArgs ha{};
    ha.key = src[1];
    ha.okey = B2[1];
    ha.nv = nv;
    for (int j = 0; j < NUT_MAX_VALS; ++j)
      if (vmap[j] >= 0) {
        ha.val[vmap[j]] = src[3 + vmap[j]];
        ha.oval[vmap[j]] = B2[3 + vmap[j]];
      }
    ha.n = n;
    ha.na = na;
    for (int a = 0; a < na; ++a) {
      ha.kind[a] = g->kinds[a];
      ha.arg[a] = s->agg_op[a] == NUT_AGG_COUNT ? 0 : vmap[s->agg_arg[a][0]];
    }
    ha.hk = (const int64_t *)dheavy;
    ha.slot = (const uint16_t *)((uint64_t *)dheavy + slot0);
    ha.seed1 = hseed1;
    ha.seed2 = hseed2;
    ha.h = nh;
    ha.hagg = (uint64_t *)dheavy + nh;
    ha.count = (uint64_t *)dheavy + nh + (size_t)nh * na;
    ha.chunk = chunk;
    c->timer.begin(st, NUT_KERNEL_AGGREGATE);
    hipLaunchKernelGGL(hkern[nv], dim3((unsigned)hgrid), dim3(HK_THREADS), 0, st, ha);
    if (exact)
      hipLaunchKernelGGL(go_cell_hist_kernel, dim3((unsigned)hgrid), dim3(GO_HIST_THREADS), 0, st, ha.okey,
                         (const uint64_t *)ha.count, chunk * HK_TILE, rg, (unsigned long long *)dheavy + cell0);
    c->timer.end(st);
    NUT_HIP(hipGetLastError());
    hcount.resize(hgrid);
    NUT_HIP(hipMemcpyAsync(hcount.data(), ha.count, hgrid * 8, hipMemcpyDeviceToHost, st));
    if (exact) {
      cells.resize(GO_CELLS);
      NUT_HIP(hipMemcpyAsync(cells.data(), dheavy + cell0, GO_CELLS * 8, hipMemcpyDeviceToHost, st));
    }
    NUT_HIP(hipStreamSynchronize(st));
    hchunk = chunk * HK_TILE;
    n0 = 0;
    for (uint64_t x : hcount) n0 += x;
    src[1] = B2[1];
    for (int j = 0; j < NUT_MAX_VALS; ++j)
      if (vmap[j] >= 0) src[3 + vmap[j]] = B2[3 + vmap[j]];
  }
  c->gb_heavy_keys = nh;
  c->gb_heavy_rows = n - n0;
  if (nh && n0 == 0) {
    // every row was a heavy key's (few distinct keys under a large group_hint): no row is
    // left for the partition levels, and the heavy pass's groups are the whole result
    // (hkeys ascending, every one seen in the data; f64 MIN / MAX back from the table order)
    std::vector<uint64_t> hw((size_t)nh * na);
    NUT_HIP(hipMemcpyAsync(hw.data(), dheavy + nh, hw.size() * 8, hipMemcpyDeviceToHost, st));
    NUT_HIP(hipStreamSynchronize(st));
    for (uint32_t j = 0; j < nh; ++j)
      for (int a = 0; a < na; ++a) {
        uint64_t &x = hw[(size_t)j * na + a];
        if (g->kinds[a] == AK_MIN_F64 || g->kinds[a] == AK_MAX_F64) x = ord_to_f64(x);
      }
    bool over = false;
    *n_out = fold_sorted_groups(keys_h, aggs_h, 0, cap, hkeys, hw, g->kinds, na, &over);
    if (over) return fail(NUT_ERR_CAPACITY, "nut_groupby_to_host: capacity " + std::to_string(cap) + " < " +
                                                std::to_string(nh) + " groups");
    return NUT_OK;
  }
  // ---- level 0 (range digit = cell >> bits1): 1.5 x the even share per partition, the rest
  // of O (~n / 2 rows) its arena
  const uint64_t ocap = ((3 * rows / 2) >> bits0) & ~1ull;
  const uint64_t abase0 = ocap << bits0, acap0 = 2 * rows - abase0 - 2 * GP_TILE;
  std::vector<GpSeg> segs;
  if (hcount.empty()) {
    segs.push_back(GpSeg{0, n, 0, 0});
  } else {  // the heavy pass's per-workgroup runs, gathered into one set of regions
    for (size_t b = 0; b < hcount.size(); ++b)
      if (hcount[b]) segs.push_back(GpSeg{b * hchunk, hcount[b], 0, 0});
    if (segs.empty()) segs.push_back(GpSeg{0, 0, 0, 0});
  }
  for (GpSeg &sg : segs) sg.ocap = ocap;
  std::vector<uint64_t> hist, p0;
  std::vector<uint32_t> dig0;  // the level-0 digit of each non-empty level-0 partition
  const uint32_t nb0 = 1u << bits0, nb1 = 1u << bits1;
  // exact: level 0 is launched after the metadata upload below (its layout is known now)
  std::vector<uint32_t> ts0;
  std::vector<uint64_t> cur0;
  if (!exact) {
    c->timer.begin(st, NUT_KERNEL_AGGREGATE);
    e = gp_level(c, mm, segs, bits1, src, O, narr, hcount.size() > 0, false, hist, &p0, 0, abase0, bits0, &rg, darena,
                 acap0);
    c->timer.end(st);
    if (e) return e == NUT_ERR_CAPACITY ? decline(NUT_GB_DECLINE_ARENA) : e;
    for (size_t i = 0; i < p0.size(); i += 2) dig0.push_back((uint32_t)(p0[i] / ocap));
  } else {
    // digit d's rows start at a 32-row boundary of O after digit d - 1's (256-B aligned)
    cur0.assign(nb0 + 1, 0);  // + the (unused) overflow flag
    uint64_t at = 0;
    for (uint32_t d = 0; d < nb0; ++d) {
      uint64_t cnt = 0;
      for (uint32_t q = 0; q < nb1; ++q) cnt += cells[(d << bits1) | q];
      cur0[d] = at;
      if (cnt) {
        p0.push_back(at);
        p0.push_back(at + cnt);
        dig0.push_back(d);
      }
      at = (at + cnt + 31) & ~31ull;
    }
    if (at + 2 * GP_TILE > 2 * rows) return decline(NUT_GB_DECLINE_CAPACITY);
    for (GpSeg &sg : segs) sg.ocap = 0;
    gp_tiles(segs, 2 * GP_TILE, ts0);
  }
  // ---- level-1 regions, as the hashed path sizes them (capped), or from the cell counts
  const uint32_t np0 = (uint32_t)(p0.size() / 2);
  std::vector<GpSeg> s2;
  uint64_t ovf1 = 0;
  for (uint32_t i = 0; i < np0; ++i) {
    GpSeg sg{p0[2 * i], p0[2 * i + 1] - p0[2 * i], 0, 0};
    sg.obase = ovf1;
    if (exact) {
      sg.ocap = 0;
      for (uint32_t q = 0; q < nb1; ++q) ovf1 += (cells[(dig0[i] << bits1) | q] + 1) & ~1ull;
    } else {
      sg.ocap = ((uint64_t)ceil((double)sg.count / nb1 * slack1) + 64 + 1) & ~1ull;
      ovf1 += sg.ocap << bits1;
    }
    s2.push_back(sg);
  }
  if (ovf1 + 2 * GP_TILE > b2rows) return decline(NUT_GB_DECLINE_CAPACITY);
  const uint64_t acap1 = b2rows - ovf1 - 2 * GP_TILE;  // level 1's arena: rows [ovf1, ovf1 + acap1) of B2
  const uint64_t nparts = (uint64_t)np0 * nb1;
  if (nparts == 0) return decline(NUT_GB_DECLINE_CAPACITY);  // (no kept row reached level 0: not reached)
  // chunks of level-0 partitions (in key order) shrinking — 3/8, 1/4, 3/16, 1/16, 1/16,
  // 1/16: a chunk's transfer (~0.4x its compute) hides behind the next, smaller chunk, and
  // only the last 1/16 crosses after the work; each launch costs a tail, so few chunks.
  // The first chunk at 3/8 instead of 1/2 starts the transfers earlier: same-box A/Bs on two
  // boxes, Zipf-like keys 17.88-17.90 vs 18.33-18.76 and 18.37-18.58 vs 19.12-19.22 ms,
  // uniform 18.21-18.24 vs 18.34-18.62 and 20.75-21.16 vs 20.90; three 1/16 chunks at the
  // end instead of 1/8 + 1/16, a third box: Zipf-like 18.42-18.56 vs 19.43-19.59, uniform
  // 20.18 vs 20.18-20.23 (profiles/r06/groupby1e7/ab_chunks.txt)
  std::vector<uint32_t> cb{0};
  for (uint32_t f : {6u, 10u, 13u, 14u, 15u, 16u}) {
    const uint32_t e1 = (uint32_t)((uint64_t)np0 * f / 16);
    if (e1 > cb.back()) cb.push_back(e1);
  }
  const uint32_t nch = (uint32_t)cb.size() - 1;
  const int l1_threads = c->opt[NUT_OPT_GB_L1_THREADS] == 512 ? 512 : 1024;  // level 1's scatter workgroup
  std::vector<uint32_t> tiles, tile0(nch + 1, 0), ntile(nch, 0);
  for (uint32_t j = 0; j < nch; ++j) {
    std::vector<GpSeg> sub(s2.begin() + cb[j], s2.begin() + cb[j + 1]);
    std::vector<uint32_t> ts;
    ntile[j] = gp_tiles(sub, (uint32_t)l1_threads * GP_ITEMS, ts);
    for (uint32_t i = 0; i < sub.size(); ++i) s2[cb[j] + i].tile0 = sub[i].tile0;
    tile0[j] = (uint32_t)tiles.size();
    tiles.insert(tiles.end(), ts.begin(), ts.end());
  }
  std::vector<uint64_t> init(nparts + nch, 0), rend(nparts);  // + one overflow flag per chunk
  for (uint32_t i = 0; i < np0; ++i) {
    uint64_t at = s2[i].obase;  // (exact: digit d's rows after digit d - 1's, even starts)
    for (uint32_t d = 0; d < nb1; ++d) {
      const uint64_t q = (uint64_t)i * nb1 + d;
      if (exact) {
        const uint64_t cnt = cells[(dig0[i] << bits1) | d];
        init[q] = at;
        rend[q] = at + cnt;
        at += (cnt + 1) & ~1ull;
      } else {
        init[q] = s2[i].obase + (uint64_t)d * s2[i].ocap;
        rend[q] = s2[i].obase + (uint64_t)(d + 1) * s2[i].ocap;
      }
    }
  }
  // the aggregation's table regions: every one holds a full block table (+ the special key)
  nut_agg_spec s3;
  memset(&s3, 0, sizeof(s3));
  s3.n = n;
  s3.nkeys = 1;
  s3.keys[0] = (const int64_t *)B2[1];
  s3.nvals = nv;
  s3.naggs = na;
  for (int j = 0; j < NUT_MAX_VALS; ++j)
    if (vmap[j] >= 0) {
      s3.val_col[vmap[j]] = B2[3 + vmap[j]];
      s3.val_type[vmap[j]] = s->val_type[j];
    }
  for (int a = 0; a < na; ++a) {
    s3.agg_op[a] = s->agg_op[a];
    s3.agg_expr[a] = NUT_EX_COL;
    if (s->agg_op[a] != NUT_AGG_COUNT) s3.agg_arg[a][0] = vmap[s->agg_arg[a][0]];
  }
  const uint64_t per = std::max<uint64_t>(64, 2 * ((group_hint + nparts - 1) / nparts));
  const uint32_t lcap = agg_lcap(c, 1, na, per, true);
  if (!lcap) return decline(NUT_GB_DECLINE_CAPACITY);
  const uint64_t dregion = (uint64_t)lcap + 1;
  if (dregion > 4097) return decline(NUT_GB_DECLINE_CAPACITY);  // (the ordering pass holds a region in LDS, <= 17 keys per thread)
  e = alloc_stage(g, nparts * dregion);
  if (e) return e;
  // device tables, uploaded once
  GpSeg *dseg;
  uint32_t *dts;
  uint64_t *dinit, *drend;
  // each heavy key's partition (heavy pass): level-0 digit -> its index among the non-empty
  // level-0 partitions (region d starts at row d * ocap), then the level-1 digit; -1: its
  // level-0 partition holds no rows (the host folds that key's group)
  std::vector<int64_t> hq(nh, -1);
  if (nh) {
    std::vector<int64_t> idx0((size_t)1 << bits0, -1);
    for (uint32_t i = 0; i < np0; ++i) idx0[dig0[i]] = i;
    for (uint32_t j = 0; j < nh; ++j) {
      const uint32_t cell = rg.cell((uint64_t)hkeys[j]);
      const int64_t i0 = idx0[cell >> bits1];
      if (i0 >= 0) hq[j] = i0 * nb1 + (cell & (nb1 - 1));
    }
  }
  e = mm.begin(GpMeta::al(s2.size() * sizeof(GpSeg)) + GpMeta::al(tiles.size() * 4 + 1) + GpMeta::al(init.size() * 8) +
               2 * GpMeta::al(init.size() * 8) + 4 * GpMeta::al(nparts * 8) + GpMeta::al(64) +
               2 * GpMeta::al((size_t)nh * 8 + 1) +
               (exact ? GpMeta::al(segs.size() * sizeof(GpSeg)) + GpMeta::al(ts0.size() * 4 + 1) +
                            GpMeta::al(cur0.size() * 8)
                      : 0));
  if (e) return e;
  if ((e = mm.up(s2, &dseg)) || (e = mm.up(tiles, &dts)) || (e = mm.up(init, &dinit)) || (e = mm.up(rend, &drend)))
    return e;
  if (exact) {  // ---- level 0 into the exact regions (no overflow check: ovf = 0)
    GpSeg *dseg0;
    uint32_t *dts0;
    uint64_t *dcur0;
    if ((e = mm.up(segs, &dseg0)) || (e = mm.up(ts0, &dts0)) || (e = mm.up(cur0, &dcur0))) return e;
    GpArrays a0;
    for (int a = 0; a < GP_MAX_ARR; ++a) {
      a0.src[a] = src[a];
      a0.dst[a] = O[a];
    }
    a0.narr = narr;
    c->timer.begin(st, NUT_KERNEL_AGGREGATE);
    gp_capped_launch(c, a0, dseg0, dts0, (uint32_t)ts0.size(), bits1, (unsigned long long *)dcur0, 0, 0,
                     (unsigned long long *)dcur0 + nb0, bits0, false, &rg, nullptr, 0, nullptr, 1);
    c->timer.end(st);
    NUT_HIP(hipGetLastError());
  }
  int64_t *dhq = nullptr;
  if ((e = mm.up(hq, &dhq))) return e;
  uint64_t *dmiss = (uint64_t *)mm.alloc((size_t)nh * 8 + 1);  // heavy keys whose partition's region was full
  if (nh) NUT_HIP(hipMemsetAsync(dmiss, 0, (size_t)nh * 8, st));
  unsigned long long *dcur = (unsigned long long *)mm.alloc(init.size() * 8);
  unsigned long long *dcount = (unsigned long long *)mm.alloc(nparts * 8);
  uint64_t *doffs = (uint64_t *)mm.alloc(nparts * 8);
  unsigned long long *drun = (unsigned long long *)mm.alloc(64);
  // the first overflowing run's start per partition (gp_scatter_kernel's acut), from the
  // region ends: the aggregation ends each partition there (AggArgs::seg_cut)
  unsigned long long *dcut = (unsigned long long *)mm.alloc(nparts * 8);
  NUT_HIP(hipMemcpyAsync(dcut, drend, nparts * 8, hipMemcpyDeviceToDevice, st));
  NUT_HIP(hipMemcpyAsync(dcur, dinit, init.size() * 8, hipMemcpyDeviceToDevice, st));
  NUT_HIP(hipMemsetAsync(drun, 0, 64, st));
  // the ordered result on the device (at most one group per row, at most cap)
  const uint64_t rcap = std::min<uint64_t>(cap, n);
  if (!c->copy_stream) NUT_HIP(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
  // released on every return, after the copy stream has drained (it reads `res` and
  // waits on the events)
  struct Cleanup {
    nut_ctx *c;
    hipStream_t st;
    uint64_t *res = nullptr;
    std::vector<hipEvent_t> ev, ev1, eva;
    ~Cleanup() {
      if (c->aux_stream) (void)hipStreamSynchronize(c->aux_stream);
      if (c->order_stream) (void)hipStreamSynchronize(c->order_stream);
      (void)hipStreamSynchronize(c->copy_stream);
      for (auto *v : {&ev, &ev1, &eva})
        for (auto x : *v)
          if (x) (void)hipEventDestroy(x);
      c->stream = st;
      if (res) (void)hipFreeAsync(res, st);
    }
  } cl{c, st};
  NUT_HIP(hipMallocAsync((void **)&cl.res, rcap * 8 * (1 + (size_t)na), st));
  int64_t *rk = (int64_t *)cl.res;
  uint64_t *ra = cl.res + rcap;
  std::vector<hipEvent_t> &ev = cl.ev;
  ev.assign(nch, nullptr);
  for (auto &x : ev) NUT_HIP(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  volatile uint64_t *runs = (volatile uint64_t *)c->host_pinned + 64;  // [nch] (pinned: 512 words)
  NUT_HIP(hipFuncSetAttribute((const void *)go_order_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)go_order_lds(dregion)));
  GpArrays ar;
  for (int a = 0; a < GP_MAX_ARR; ++a) {
    ar.src[a] = O[a];
    ar.dst[a] = B2[a];
  }
  ar.narr = narr;
  // Four streams: level 1 of every chunk back to back on the context's stream; each
  // chunk's aggregation on a second one as soon as its level 1 is done (it overlaps the
  // next chunk's level 1, so neither launch's tail idles the chip); its ordering on a third
  // as soon as its aggregation is done; its transfer on the fourth once the host has read
  // the chunk's running total.  (With the runtime's four hardware queues the third stream
  // lands on the aggregation's queue, so orderings and aggregations still alternate; the
  // ordering on a high-priority stream, a queue of its own, ran beside them and stretched
  // all three: 20.4 vs 19.3 ms per G = 1e7 step, profiles/r06/groupby1e7/ab_order_priority.txt)
  if (!c->aux_stream) NUT_HIP(hipStreamCreateWithFlags(&c->aux_stream, hipStreamNonBlocking));
  if (!c->order_stream) NUT_HIP(hipStreamCreateWithFlags(&c->order_stream, hipStreamNonBlocking));
  hipStream_t ax = c->aux_stream, ox = c->order_stream;
  std::vector<hipEvent_t> &ev1 = cl.ev1, &eva = cl.eva;
  ev1.assign(nch, nullptr);
  eva.assign(nch, nullptr);
  for (auto &x : ev1) NUT_HIP(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  for (auto &x : eva) NUT_HIP(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  auto enqueue = [&](uint32_t j) -> nut_status {
    const uint32_t a0 = cb[j], a1 = cb[j + 1];
    const uint64_t q0 = (uint64_t)a0 * nb1, nq = (uint64_t)(a1 - a0) * nb1;
    c->timer.begin(st, NUT_KERNEL_AGGREGATE);
    gp_capped_launch(c, ar, dseg + a0, dts + tile0[j], ntile[j], 0, dcur + q0, 0, exact ? 0 : ovf1, dcur + nparts + j,
                     bits1, false, &rg, exact ? nullptr : darena + 1, acap1, exact ? nullptr : dcut + q0, 0,
                     l1_threads, j ? (int)c->opt[NUT_OPT_GB_L1_SPARE] : 0);
    c->timer.end(st);
    NUT_HIP(hipGetLastError());
    NUT_HIP(hipEventRecord(ev1[j], st));
    NUT_HIP(hipStreamWaitEvent(ax, ev1[j], 0));
    // partition rows [first row, cursor after the scatter), cut at the first run that went
    // to the arena (the rows after it are not the partition's): min(cursor, cut), read by
    // the aggregation's blocks themselves
    LaunchExtra sg;
    sg.seg_off = dinit + q0;
    sg.seg_end = (const uint64_t *)dcur + q0;
    sg.seg_cut = (const uint64_t *)dcut + q0;
    sg.nseg = (uint32_t)nq;
    sg.dense = true;
    sg.dcount = dcount + q0;
    sg.dregion = dregion;
    sg.dbase = q0;
    c->stream = ax;  // (launch_agg launches on the context's stream)
    nut_status e2 = launch_agg(g, &s3, per, g->kinds, &sg);
    c->stream = st;
    if (e2) return e2;
    if (nh)  // the heavy keys' groups of this chunk's partitions join their regions before the ordering
      hipLaunchKernelGGL(go_heavy_insert_kernel, dim3(1), dim3(1024), 0, ax, (const int64_t *)dheavy,
                         (const uint64_t *)dheavy + nh, nh, na, (const int64_t *)dhq, q0, nq, dcount, g->gt.slot,
                         g->gt.agg, g->gt.cap + 1, dregion, dmiss);
    NUT_HIP(hipEventRecord(eva[j], ax));
    NUT_HIP(hipStreamWaitEvent(ox, eva[j], 0));
    c->timer.begin(ox, NUT_KERNEL_AGGREGATE);
    hipLaunchKernelGGL(go_scan_kernel, dim3(1), dim3(1024), 0, ox, (const unsigned long long *)dcount + q0, (uint32_t)nq,
                       doffs + q0, drun);
    hipLaunchKernelGGL(go_order_kernel, dim3((unsigned)nq), dim3(GO_ORDER_THREADS), (unsigned)go_order_lds(dregion), ox,
                       (const uint64_t *)g->gt.slot, (const uint64_t *)g->gt.agg, g->gt.cap + 1, dregion, q0,
                       (const unsigned long long *)dcount + q0, (const uint64_t *)doffs + q0, na, g->gt.kinds, rk, ra,
                       rcap);
    c->timer.end(ox);
    NUT_HIP(hipGetLastError());
    NUT_HIP(hipMemcpyAsync((void *)(runs + j), drun, 8, hipMemcpyDeviceToHost, ox));
    NUT_HIP(hipEventRecord(ev[j], ox));
    return NUT_OK;
  };
  // every chunk queued (nothing waits for the host); chunk j crosses on the copy stream
  // once its count is known
  uint64_t done = 0;  // groups already sent to the host
  bool over = false;
  for (uint32_t j = 0; j < nch; ++j)
    if ((e = enqueue(j))) return e;
  for (uint32_t j = 0; j < nch; ++j) {
    NUT_HIP(hipEventSynchronize(ev[j]));
    const uint64_t total = runs[j];
    if (total > rcap) over = true;
    if (!over && total > done) {
      NUT_HIP(hipStreamWaitEvent(c->copy_stream, ev[j], 0));
      NUT_HIP(hipMemcpyAsync(keys_h + done, rk + done, (total - done) * 8, hipMemcpyDeviceToHost, c->copy_stream));
      NUT_HIP(hipMemcpyAsync(aggs_h + done * na, ra + done * na, (total - done) * 8 * na, hipMemcpyDeviceToHost,
                             c->copy_stream));
    }
    done = total;
  }
  // the capped level-1 flags (an exhausted arena), the arenas' fill and the aggregation's
  // control words
  NUT_HIP(hipStreamSynchronize(ax));
  NUT_HIP(hipStreamSynchronize(ox));
  // (everything in gp_meta is read now: the arenas' group-by below may partition, and its
  // own tables take gp_meta)
  std::vector<uint64_t> flags(nch), miss(nh);
  NUT_HIP(hipMemcpyAsync(flags.data(), dcur + nparts, nch * 8, hipMemcpyDeviceToHost, st));
  if (nh) NUT_HIP(hipMemcpyAsync(miss.data(), dmiss, (size_t)nh * 8, hipMemcpyDeviceToHost, st));
  uint32_t ctl[4];
  NUT_HIP(hipMemcpyAsync(c->host_pinned, g->gt.ctl, 16, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipMemcpyAsync(c->host_pinned + 2, darena, 16, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipStreamSynchronize(st));
  memcpy(ctl, c->host_pinned, 16);
  const uint64_t used0 = c->host_pinned[2], used1 = c->host_pinned[3];
  NUT_HIP(hipStreamSynchronize(c->copy_stream));
  for (uint64_t f : flags)
    if (f) return decline(NUT_GB_DECLINE_ARENA);  // a level-1 run found the arena full
  if (ctl[1] & 4u) return decline(NUT_GB_DECLINE_TABLE);  // a partition outgrew its block's table
  c->gb_overflow_rows = used0 + used1;
  if (used0 + used1 && !over) {
    // the arenas' rows (heavy keys' excess, mostly) aggregated on their own and folded
    // into the ordered host result
    // (copied out of gp_data first — the arenas live there and the group-by may partition,
    // which takes gp_data — then one group-by over both levels' rows, on whichever path its
    // size picks)
    const uint64_t ar_rows = used0 + used1, ar_str = (ar_rows + 31) & ~31ull;  // (arrays 256-B aligned: vector loads)
    uint64_t *ar = nullptr;
    NUT_HIP(hipMallocAsync((void **)&ar, ar_str * 8 * (1 + (size_t)nv), st));
    struct FreeAr {
      uint64_t *p;
      hipStream_t s;
      ~FreeAr() { (void)hipFreeAsync(p, s); }
    } free_ar{ar, st};
    for (int i = 1; i < narr; ++i) {
      if (i == 2) continue;
      uint64_t *dst = ar + (size_t)(i == 1 ? 0 : i - 2) * ar_str;
      if (used0) NUT_HIP(hipMemcpyAsync(dst, O[i] + abase0, used0 * 8, hipMemcpyDeviceToDevice, st));
      if (used1) NUT_HIP(hipMemcpyAsync(dst + used0, B2[i] + ovf1, used1 * 8, hipMemcpyDeviceToDevice, st));
    }
    nut_agg_spec sa = s3;
    sa.n = ar_rows;
    sa.keys[0] = (const int64_t *)ar;
    for (int j = 0; j < NUT_MAX_VALS; ++j)
      if (vmap[j] >= 0) sa.val_col[vmap[j]] = ar + (size_t)(1 + vmap[j]) * ar_str;
    // (partitioned whatever its size: the rows are the tails of many keys — up to one group
    // per row — and the streaming path's global table would take every one of them by
    // atomics: 4 ms for 8.7 M arena rows of the 1e9-row Zipf step)
    const uint32_t path = c->gb_path, lv = c->gb_levels, opt = c->gb_optimistic;
    const int64_t part = c->opt[NUT_OPT_GB_PARTITION];
    c->opt[NUT_OPT_GB_PARTITION] = 1;
    nut_groups *ga = nullptr;
    uint64_t na_groups = 0;
    e = nut_groupby(c, &sa, std::min<uint64_t>(ar_rows, group_hint), &ga);
    c->opt[NUT_OPT_GB_PARTITION] = part;
    c->gb_path = path, c->gb_levels = lv, c->gb_optimistic = opt;
    if (!e) e = nut_groups_size(ga, &na_groups);
    std::vector<int64_t> hk(na_groups);
    std::vector<uint64_t> hw(na_groups * (size_t)na);
    if (!e && na_groups) e = nut_groups_to_host(ga, hk.data(), hw.data(), na_groups);
    nut_groups_free(ga);
    if (e) return e;
    done = fold_sorted_groups(keys_h, aggs_h, done, cap, hk, hw, g->kinds, na, &over);
  }
  if (nh && !over) {
    // heavy keys that joined no region (their level-0 partition was empty, or the region
    // was full): folded here (result words: f64 MIN / MAX back from the table order)
    std::vector<uint64_t> hw((size_t)nh * na);
    NUT_HIP(hipMemcpyAsync(hw.data(), dheavy + nh, hw.size() * 8, hipMemcpyDeviceToHost, st));
    NUT_HIP(hipStreamSynchronize(st));
    std::vector<int64_t> fk;
    std::vector<uint64_t> fw;
    for (uint32_t j = 0; j < nh; ++j) {
      if (hq[j] >= 0 && !miss[j]) continue;
      fk.push_back(hkeys[j]);
      for (int a = 0; a < na; ++a) {
        const uint64_t x = hw[(size_t)j * na + a];
        fw.push_back(g->kinds[a] == AK_MIN_F64 || g->kinds[a] == AK_MAX_F64 ? ord_to_f64(x) : x);
      }
    }
    if (!fk.empty()) done = fold_sorted_groups(keys_h, aggs_h, done, cap, fk, fw, g->kinds, na, &over);
  }
  *n_out = done;
  if (over) return fail(NUT_ERR_CAPACITY, "nut_groupby_to_host: capacity " + std::to_string(cap) + " < " +
                                              std::to_string(done) + " groups");
  return NUT_OK;
}

// Spill -> partition -> per-partition aggregation into g's table.  *used = false when the
// query does not fit the staged layout (more than NUT_MAX_VALS staged value arrays).
nut_status groupby_partitioned(nut_groups *g, const nut_agg_spec *s, uint64_t group_hint, bool *used) {
  *used = false;
  nut_ctx *c = g->ctx;
  hipStream_t st = c->stream;
  const int nk = g->nk, na = g->naggs;
  // staged value arrays: every aggregate except a COUNT that takes every row
  LaunchExtra sp;
  sp.spill = true;
  int32_t kinds2[NUT_MAX_AGGS];
  int nv = 0;
  for (int a = 0; a < na; ++a) {
    const bool masked = s->prog_mode && s->agg_mask[a].n;
    const bool need = g->kinds[a] != AK_COUNT || masked;
    sp.sp_map[a] = need ? nv++ : -1;
    kinds2[a] = g->kinds[a] == AK_COUNT && need ? AK_SUM_I64 : g->kinds[a];
  }
  if (nv > NUT_MAX_VALS) return NUT_OK;
  *used = true;
  // Direct path: no WHERE and every argument a plain column (BASELINE config 3) — the
  // spill would only copy the key and value columns, so the first partition level reads
  // them in place (a key histogram pass of 8 B/row instead of a 32 B/row spill).
  bool direct = !s->prog_mode && s->npred == 0 && c->opt[NUT_OPT_GB_DIRECT] != 0;
  for (int a = 0; a < na && direct; ++a) direct = s->agg_op[a] == NUT_AGG_COUNT || s->agg_expr[a] == NUT_EX_COL;
  if (direct) return groupby_partitioned_direct(g, s, group_hint);
  const int narr = 3 + nv;  // -, k1, k2 (unused for one key), values
  const uint64_t n = s->n;
  // staging: every block's region (<= n + one region of slack per block) in A, the
  // compact partitioned records in B (and A again after a second level)
  const uint64_t maxblocks = (uint64_t)c->num_cus * 8;
  // (+ one alignment gap per final partition; a multiple of 32 keeps every array 256-B aligned)
  const uint64_t rows = (n + maxblocks * 2 * kBdShared + 2 * 65536 + 64 + 31) & ~31ull;
  const int nstore = narr - 1 - (nk == 1 ? 1 : 0);  // k1, [k2], values
  nut_status e = c->gp_data.reserve(2 * (size_t)nstore * rows * 8 + 256);
  if (e) return e;
  uint64_t *A[GP_MAX_ARR] = {}, *B[GP_MAX_ARR] = {};
  for (int i = 1, k = 0; i < narr; ++i) {
    if (i == 2 && nk == 1) continue;
    A[i] = (uint64_t *)c->gp_data.ptr + (size_t)k * rows;
    B[i] = (uint64_t *)c->gp_data.ptr + (size_t)(nstore + k) * rows;
    ++k;
  }
  GpMeta mm{c};
  // ---- 1. spill: WHERE + aggregate arguments evaluated, rows staged per block in A
  e = mm.begin(GpMeta::al(maxblocks * 8) + GpMeta::al(GP_BINS * 8));
  if (e) return e;
  unsigned long long *dcnt = (unsigned long long *)mm.alloc(maxblocks * 8);
  unsigned long long *dh0 = (unsigned long long *)mm.alloc(GP_BINS * 8);
  NUT_HIP(hipMemsetAsync(dh0, 0, GP_BINS * 8, st));
  sp.sp_counts = dcnt;
  sp.sp_hist = dh0;
  for (int i = 1; i < narr; ++i) sp.sp_cols[i] = A[i];
  e = launch_agg(g, s, group_hint, g->kinds, &sp);
  if (e) return e;
  std::vector<uint64_t> cnt(sp.blocks), hist(GP_BINS);
  NUT_HIP(hipMemcpyAsync(cnt.data(), dcnt, sp.blocks * 8, hipMemcpyDeviceToHost, st));
  NUT_HIP(hipMemcpyAsync(hist.data(), dh0, GP_BINS * 8, hipMemcpyDeviceToHost, st));
  uint32_t ctl[4];
  e = read_ctl(g, ctl);
  if (e) return e;
  if (ctl[1] & 2u) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: division by zero in an expression");
  std::vector<GpSeg> segs;
  uint64_t nsp = 0;
  for (uint64_t b = 0; b < sp.blocks; ++b) {
    if (cnt[b]) segs.push_back(GpSeg{b * sp.region, cnt[b], 0, 0});
    nsp += cnt[b];
  }
  if (nsp == 0) return NUT_OK;
  // ---- 2. partition by the key hash: 256 or 65536 partitions of ~<= 1K groups
  const int levels = c->opt[NUT_OPT_GB_LEVELS] ? (int)c->opt[NUT_OPT_GB_LEVELS] : group_hint > 256ull * 1024 ? 2 : 1;
  c->gb_path = NUT_GB_PARTITIONED_SPILL;
  c->gb_levels = (uint32_t)levels;
  c->gb_optimistic = 0;
  c->timer.begin(st, NUT_KERNEL_AGGREGATE);
  std::vector<uint64_t> parts;  // [start, end) pairs of the final partitions
  uint64_t **fin = B;
  if (levels == 1) {
    e = gp_level(c, mm, segs, 56, A, B, narr, true, true, hist, &parts);
    if (e) return e;
  } else {
    e = gp_level(c, mm, segs, 56, A, B, narr, true, true, hist);
    if (e) return e;
    std::vector<GpSeg> s2;
    uint64_t run = 0;
    for (int d = 0; d < GP_BINS; ++d) {
      if (hist[d]) s2.push_back(GpSeg{run, hist[d], 0, 0});
      run += hist[d];
    }
    std::vector<uint64_t> h2;
    e = gp_level(c, mm, s2, 48, B, A, narr, false, false, h2, &parts);
    if (e) return e;
    fin = A;
  }
  c->timer.end(st);
  // ---- 3. one workgroup per partition, its groups in LDS, merged into g's table once
  nut_agg_spec s2;
  memset(&s2, 0, sizeof(s2));
  s2.n = nsp;  // (segment mode reads only the listed ranges)
  s2.nkeys = nk;
  s2.keys[0] = (const int64_t *)fin[1];
  s2.keys[1] = nk == 2 ? (const int64_t *)fin[2] : nullptr;
  s2.nvals = nv;
  s2.naggs = na;
  for (int a = 0; a < na; ++a) {
    const int k = kinds2[a];
    s2.agg_op[a] = k == AK_COUNT ? NUT_AGG_COUNT : (k == AK_SUM_F64 || k == AK_SUM_I64) ? NUT_AGG_SUM
                   : (k == AK_MIN_F64 || k == AK_MIN_I64) ? NUT_AGG_MIN : NUT_AGG_MAX;
    s2.agg_expr[a] = NUT_EX_COL;
    if (sp.sp_map[a] >= 0) {
      s2.agg_arg[a][0] = sp.sp_map[a];
      s2.val_col[sp.sp_map[a]] = fin[3 + sp.sp_map[a]];
      s2.val_type[sp.sp_map[a]] = (k == AK_SUM_F64 || k == AK_MIN_F64 || k == AK_MAX_F64) ? NUT_T_F64 : NUT_T_I64;
    }
  }
  return gp_aggregate(g, mm, parts, s2, kinds2, group_hint);
}

}  // namespace

extern "C" {

// NUT_OPT_PRIV_PROBE: before the first compiled-Q1-shape launch of >= 2^27 rows on a
// device, time the kernel at each of kPrivShapes over the caller's whole input (two
// interleaved rounds, best of each; the kernel timer is paused, so no probe launch is
// counted as the caller's work) and keep the fastest for the device — another shape than
// the default 192 x 2 only if it is >= 0.5 % faster (the shapes lie within ~1 % of each other
// and a 2^28-row slice had picked 128 x 3 where the full-size table, same box, had 192 x 2
// ahead: 7.447 vs 7.502 ms, profiles/r05/q1/probe_full_size.txt).  The probe launches fold
// into g's table, which is initialised again afterwards: the result is the real launch's
// alone.
static nut_status probe_priv_shape(nut_groups *g, const nut_agg_spec *s, uint64_t group_hint, uint64_t cap) {
  nut_ctx *c = g->ctx;
  if (!c->opt[NUT_OPT_PRIV_PROBE] || c->opt[NUT_OPT_PRIV_BD] || c->opt[NUT_OPT_PRIV_BLOCKS] || s->n < (1ull << 27) ||
      c->device < 0 || c->device >= 64 || priv_shape_of(c->device).shape >= 0)
    return NUT_OK;
  LaunchExtra dry;
  dry.dry = true;
  nut_status st = launch_agg(g, s, group_hint, g->kinds, &dry);
  if (st || !dry.q1_fused) return st;
  nut_agg_spec s2 = *s;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  NUT_HIP(hipEventCreate(&e0));
  hipError_t he = hipEventCreate(&e1);
  if (he != hipSuccess) {
    (void)hipEventDestroy(e0);
    return hip_fail(he, "hipEventCreate");
  }
  const bool timing = c->timer.enabled;
  c->timer.enabled = false;
  const auto t0 = std::chrono::steady_clock::now();
  double best[3] = {1e30, 1e30, 1e30};
  for (int rep = 0; rep < 2 && !st; ++rep)
    for (int k = 0; k < 3 && !st; ++k) {
      c->priv_probe = k;
      he = hipEventRecord(e0, c->stream);
      if (he == hipSuccess) st = launch_agg(g, &s2, group_hint, g->kinds);
      if (he == hipSuccess && !st) he = hipEventRecord(e1, c->stream);
      if (he == hipSuccess && !st) he = hipEventSynchronize(e1);
      float ms = 0;
      if (he == hipSuccess && !st) he = hipEventElapsedTime(&ms, e0, e1);
      if (he != hipSuccess && !st) st = hip_fail(he, "nut_groupby (launch-shape probe)");
      best[k] = std::min(best[k], (double)ms);
    }
  c->priv_probe = -1;
  c->timer.enabled = timing;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (st) return st;
  int k = 0;
  for (int j = 1; j < 3; ++j)
    if (best[j] < best[k] && best[j] < 0.995 * best[0]) k = j;
  {
    std::lock_guard<std::mutex> lk(g_priv_mu);
    g_priv_shape[c->device].shape = k;
    for (int j = 0; j < 3; ++j) g_priv_shape[c->device].ms[j] = best[j];
    g_priv_shape[c->device].cost_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return alloc_table(g, cap);  // the probe's partial groups are discarded
}

nut_status nut_ctx_groupby_overflow(nut_ctx *c, uint64_t *rows, uint32_t *declined) {
  if (!c) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_groupby_overflow: NULL context");
  if (rows) *rows = c->gb_overflow_rows;
  if (declined) *declined = c->gb_decline;
  return NUT_OK;
}

nut_status nut_ctx_groupby_heavy(nut_ctx *c, uint32_t *keys, uint64_t *rows) {
  if (!c) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_groupby_heavy: NULL context");
  if (keys) *keys = c->gb_heavy_keys;
  if (rows) *rows = c->gb_heavy_rows;
  return NUT_OK;
}

nut_status nut_ctx_priv_shape(nut_ctx *c, int *threads, int *blocks_per_cu, double probe_ms[3]) {
  if (!c) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_priv_shape: NULL context");
  const PrivShape p = priv_shape_of(c->device);
  const int k = p.shape >= 0 ? p.shape : 0;
  if (threads) *threads = c->opt[NUT_OPT_PRIV_BD] ? (int)c->opt[NUT_OPT_PRIV_BD] : kPrivShapes[k][0];
  if (blocks_per_cu) *blocks_per_cu = c->opt[NUT_OPT_PRIV_BLOCKS] ? (int)c->opt[NUT_OPT_PRIV_BLOCKS] : kPrivShapes[k][1];
  if (probe_ms)
    for (int j = 0; j < 3; ++j) probe_ms[j] = p.ms[j];
  return NUT_OK;
}

nut_status nut_ctx_priv_probe_cost(nut_ctx *c, double *ms) {
  if (!c || !ms) return fail(NUT_ERR_INVALID_ARG, "nut_ctx_priv_probe_cost: NULL argument");
  *ms = priv_shape_of(c->device).cost_ms;
  return NUT_OK;
}

nut_status nut_groupby(nut_ctx *c, const nut_agg_spec *s, uint64_t group_hint, nut_groups **out) {
  if (!c || !out) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: NULL argument");
  *out = nullptr;
  nut_status st = validate(s);
  if (st) return st;
  DeviceGuard dg(c->device);
  nut_groups *g = new nut_groups();
  g->ctx = c;
  g->nk = s->nkeys ? s->nkeys : 1;  // a global aggregate is one group with key 0
  g->naggs = s->naggs;
  for (int a = 0; a < s->naggs; ++a) g->kinds[a] = kind_of(s, a);
  if (s->nkeys == 0) group_hint = 1;
  uint64_t cap = table_cap_for(group_hint ? group_hint : 8192);
  const int64_t gp = c->opt[NUT_OPT_GB_PARTITION];
  c->gb_path = NUT_GB_ONCHIP;
  c->gb_levels = c->gb_optimistic = 0;
  if (s->nkeys >= 1 && s->n && gp != 0 && (gp == 1 || (group_hint >= kGpMinGroups && s->n >= 4 * group_hint))) {
    bool used = false;
    st = alloc_table(g, cap);
    if (!st) st = groupby_partitioned(g, s, group_hint, &used);
    if (st) {
      nut_groups_free(g);
      return st;
    }
    if (used) {
      *out = g;
      return NUT_OK;
    }
  }
  for (int attempt = 0;; ++attempt) {
    st = alloc_table(g, cap);
    if (!st && attempt == 0) st = probe_priv_shape(g, s, group_hint, cap);
    if (!st) st = launch_agg(g, s, group_hint, g->kinds);
    uint32_t ctl[4] = {0, 0, 0, 0};
    if (!st) st = read_ctl(g, ctl);
    if (st) {
      nut_groups_free(g);
      return st;
    }
    if (ctl[1] & 2u) {
      nut_groups_free(g);
      return fail(NUT_ERR_INVALID_ARG, "nut_groupby: division by zero in an expression");
    }
    if (!(ctl[1] & 1u)) break;
    // more groups than the table admits: retry with a larger table
    if (cap >= (1ull << 34) || attempt > 12) {
      nut_groups_free(g);
      return fail(NUT_ERR_OOM, "nut_groupby: group table would exceed device memory");
    }
    cap *= 4;
    group_hint = std::max<uint64_t>(group_hint, ctl[0]);
  }
  *out = g;
  return NUT_OK;
}

nut_status nut_groupby_accumulate(nut_ctx *c, const nut_agg_spec *s, nut_groups *g) {
  if (!c || !g) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_accumulate: NULL argument");
  nut_status st = validate(s);
  if (st) return st;
  if ((s->nkeys ? s->nkeys : 1) != g->nk || s->naggs != g->naggs)
    return fail(NUT_ERR_INVALID_ARG, "nut_groupby_accumulate: spec shape differs from the result");
  int32_t kinds[NUT_MAX_AGGS];
  for (int a = 0; a < s->naggs; ++a) {
    int32_t k = kind_of(s, a);
    bool same = k == g->kinds[a] || (g->kinds[a] == AK_COUNT && k == AK_SUM_I64);
    if (!same) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_accumulate: aggregate kinds differ");
    kinds[a] = g->kinds[a] == AK_COUNT ? AK_SUM_I64 : k;  // COUNT partials merge by addition
  }
  DeviceGuard dg(c->device);
  g->ctx = c;
  st = ensure_room(g, s->n);
  if (st) return st;
  st = launch_agg(g, s, s->n, kinds);
  if (st) return st;
  uint32_t ctl[4];
  st = read_ctl(g, ctl);
  if (st) return st;
  if (ctl[1] & 2u) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_accumulate: division by zero in an expression");
  if (ctl[1]) return fail(NUT_ERR_OOM, "nut_groupby_accumulate: table overflow");
  return NUT_OK;
}

nut_status nut_groups_size(nut_groups *g, uint64_t *n) {
  if (!g || !n) return fail(NUT_ERR_INVALID_ARG, "nut_groups_size: NULL argument");
  DeviceGuard dg(g->ctx->device);
  uint32_t ctl[4];
  nut_status st = read_ctl(g, ctl);
  if (st) return st;
  *n = (uint64_t)ctl[0] + (g->nk == 1 && ctl[2] ? 1 : 0);
  return NUT_OK;
}

nut_status nut_groups_to_device(nut_groups *g, uint64_t *out, uint64_t cap) {
  if (!g) return fail(NUT_ERR_INVALID_ARG, "nut_groups_to_device: NULL argument");
  uint64_t n;
  nut_status st = nut_groups_size(g, &n);
  if (st) return st;
  if (n > cap)
    return fail(NUT_ERR_CAPACITY, "nut_groups_to_device: capacity " + std::to_string(cap) + " < " +
                                      std::to_string(n) + " groups");
  if (n == 0) return NUT_OK;
  if (!out) return fail(NUT_ERR_INVALID_ARG, "nut_groups_to_device: NULL output");
  nut_ctx *c = g->ctx;
  DeviceGuard dg(c->device);
  NUT_HIP(hipMemsetAsync(g->dev_cursors, 0, 64 * 8, c->stream));
  uint64_t stride = g->gt.cap + 1;
  uint64_t blocks = std::min<uint64_t>((stride + GT_CHUNK - 1) / GT_CHUNK, (uint64_t)c->num_cus * 8);
  hipLaunchKernelGGL(gtable_compact_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream,
                     (const GTable *)g->dev_gt, g->nk, out, n, g->dev_cursors, 1, (const uint64_t *)nullptr);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

nut_status nut_groups_partition(nut_groups *g, int nparts, uint64_t *out, uint64_t cap, uint64_t *counts) {
  if (!g || !counts || nparts < 1 || nparts > 64) return fail(NUT_ERR_INVALID_ARG, "nut_groups_partition: bad argument");
  nut_ctx *c = g->ctx;
  DeviceGuard dg(c->device);
  uint64_t n;
  nut_status st = nut_groups_size(g, &n);
  if (st) return st;
  if (n > cap) return fail(NUT_ERR_CAPACITY, "nut_groups_partition: capacity too small");
  if (nparts == 1) {
    counts[0] = n;
    return nut_groups_to_device(g, out, cap);
  }
  uint64_t stride = g->gt.cap + 1;
  uint64_t blocks = std::min<uint64_t>((stride + GT_CHUNK - 1) / GT_CHUNK, (uint64_t)c->num_cus * 8);
  NUT_HIP(hipMemsetAsync(g->dev_cursors, 0, 64 * 8, c->stream));
  hipLaunchKernelGGL(gtable_owner_count_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream,
                     (const GTable *)g->dev_gt, g->nk, nparts, g->dev_cursors);
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipMemcpyAsync(c->host_pinned, g->dev_cursors, 8 * nparts, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  uint64_t seg[128];
  uint64_t run = 0;
  for (int p = 0; p < nparts; ++p) {
    counts[p] = c->host_pinned[p];
    seg[p] = run;
    seg[nparts + p] = counts[p];
    run += counts[p];
  }
  if (run == 0) return NUT_OK;
  if (!out) return fail(NUT_ERR_INVALID_ARG, "nut_groups_partition: NULL output");
  NUT_HIP(hipMemcpyAsync(g->dev_segbase, seg, 16 * nparts, hipMemcpyHostToDevice, c->stream));
  NUT_HIP(hipMemsetAsync(g->dev_cursors, 0, 64 * 8, c->stream));
  hipLaunchKernelGGL(gtable_compact_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream,
                     (const GTable *)g->dev_gt, g->nk, out, run, g->dev_cursors, nparts,
                     (const uint64_t *)g->dev_segbase);
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipStreamSynchronize(c->stream));
  return NUT_OK;
}

nut_status nut_groupby_jit_source(const nut_agg_spec *s, char *buf, size_t cap, size_t *len) {
  nut_status st = validate(s);
  if (st) return st;
  if (!s->prog_mode) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_jit_source: spec is not in expression mode");
  int32_t kinds[NUT_MAX_AGGS];
  for (int a = 0; a < s->naggs; ++a) kinds[a] = kind_of(s, a);
  JitShape js;
  st = jit_shape(s, kinds, js);
  if (st) return st;
  if (len) *len = js.src.size();
  if (buf && cap) {
    size_t k = std::min(cap - 1, js.src.size());
    memcpy(buf, js.src.data(), k);
    buf[k] = '\0';
  }
  return cap && js.src.size() >= cap ? fail(NUT_ERR_CAPACITY, "nut_groupby_jit_source: buffer too small") : NUT_OK;
}

nut_status nut_groupby_jit_compile(const nut_agg_spec *s) {
  nut_status st = validate(s);
  if (st) return st;
  if (!s->prog_mode) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_jit_compile: spec is not in expression mode");
  int32_t kinds[NUT_MAX_AGGS];
  for (int a = 0; a < s->naggs; ++a) kinds[a] = kind_of(s, a);
  JitShape js;
  st = jit_shape(s, kinds, js);
  if (st) return st;
  return jit_kernel(jit_unit(js.src, s->nkeys == 2 ? 2 : 1, false, kBdShared, sizeof(AggArgs)), false, nullptr);
}

}  // extern "C"

namespace nut {
// Row i of the compacted columns goes to its key's rank among the (unique, sorted) keys:
// keys_out[rank] = key, aggs_out[rank * naggs + a] = aggregate a.
// Bucket index over the sorted unique keys (n >= 2): bucket(k) = (k - sorted[0]) >> shift,
// at most 2^PL_BITS + 1 buckets; start[b] = the first i with bucket(sorted[i]) >= b, for
// b in [0, nb].  A group then binary-searches only its bucket's run (a few keys, one or two
// cache lines) instead of the whole array (~12 random HBM lines per key at 1e7 groups).
constexpr int PL_BITS = 20;
struct PlaceBuckets {
  uint64_t mn;
  int shift;
  uint64_t nb;  // buckets 0 .. nb - 1
};
__device__ __forceinline__ PlaceBuckets place_buckets(const int64_t *sorted, uint64_t n) {
  const uint64_t mn = (uint64_t)sorted[0], range = (uint64_t)sorted[n - 1] - mn;
  const int hb = range ? 64 - __builtin_clzll(range) : 0;
  const int shift = hb > PL_BITS ? hb - PL_BITS : 0;
  return PlaceBuckets{mn, shift, (range >> shift) + 1};
}

__global__ void place_index_kernel(const int64_t *__restrict__ sorted, uint64_t n, uint64_t *__restrict__ start) {
  const PlaceBuckets pb = place_buckets(sorted, n);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b0 = i == 0 ? 0 : (((uint64_t)sorted[i - 1] - pb.mn) >> pb.shift) + 1;
    const uint64_t b1 = i == n ? pb.nb : (((uint64_t)sorted[i] - pb.mn) >> pb.shift);
    for (uint64_t b = b0; b <= b1; ++b) start[b] = i;
  }
}

__global__ void groups_place_kernel(const uint64_t *__restrict__ cols, const int64_t *__restrict__ sorted, uint64_t n,
                                    int naggs, int64_t *__restrict__ keys_out, uint64_t *__restrict__ aggs_out,
                                    const uint64_t *__restrict__ start) {
  const PlaceBuckets pb = place_buckets(sorted, n);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t k = (int64_t)cols[i];
    const uint64_t b = ((uint64_t)k - pb.mn) >> pb.shift;
    uint64_t lo = start[b], len = start[b + 1] - lo;
    while (len > 0) {  // lower bound within the bucket
      const uint64_t half = len >> 1;
      if (sorted[lo + half] < k) {
        lo += half + 1;
        len -= half + 1;
      } else {
        len = half;
      }
    }
    keys_out[lo] = k;
    for (int a = 0; a < naggs; ++a) aggs_out[lo * naggs + a] = cols[(uint64_t)(1 + a) * n + i];
  }
}

__global__ void iota_kernel(int64_t *__restrict__ out, uint64_t n, int64_t base) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = base + (int64_t)i;
}
}  // namespace nut

extern "C" {

// Expression-mode scan (select_kernel.hpp): the row ids where the spec's WHERE program
// holds, in row order.  Reads s->n, s->where and the program columns only.
nut_status nut_select_rows(nut_ctx *c, const nut_agg_spec *s, int64_t *out_rows, uint64_t *count_host) {
  if (!c || !s || !count_host || (s->n && !out_rows)) return fail(NUT_ERR_INVALID_ARG, "nut_select_rows: NULL argument");
  if (!s->prog_mode) return fail(NUT_ERR_INVALID_ARG, "nut_select_rows: needs an expression-mode spec (prog_mode = 1)");
  if (s->nprog_cols < 0 || s->nprog_cols > NUT_MAX_PROG_COLS)
    return fail(NUT_ERR_INVALID_ARG, "nut_select_rows: bad program column count");
  *count_host = 0;
  for (int i = 0; i < s->nprog_cols; ++i)
    if (s->n && !s->prog_col[i]) return fail(NUT_ERR_INVALID_ARG, "nut_select_rows: NULL program column");
  nut_agg_spec q = *s;  // the WHERE program alone
  q.naggs = 0;
  int32_t kinds[NUT_MAX_AGGS] = {};
  JitShape js;
  nut_status st = jit_shape(&q, kinds, js);
  if (st) return st;
  if (js.consts.size() > (size_t)kMaxConst)
    return fail(NUT_ERR_UNSUPPORTED, "nut_select_rows: more than 64 distinct expression constants");
  if (s->n == 0) return NUT_OK;
  const uint64_t n = s->n;
  const uint64_t ntiles = (n + SEL_TILE - 1) / SEL_TILE;
  if (ntiles > 0xFFFFFFF0ull) return fail(NUT_ERR_UNSUPPORTED, "nut_select_rows: n too large");
  DeviceGuard dg(c->device);
  hipFunction_t fn;
  st = jit_kernel(jit_select_unit(js.src, sizeof(SelArgs)), true, &fn);
  if (st) return st;
  // [ticket u32, err u32, out_n u64][status u64 x ntiles], zeroed as one block
  const size_t state = 16 + ntiles * 8;
  st = c->filter_state.reserve(state);
  if (st) return st;
  char *base = (char *)c->filter_state.ptr;
  SelArgs sa;
  memset(&sa, 0, sizeof sa);
  sa.a.n = n;
  sa.a.nvals = s->nprog_cols;
  for (int i = 0; i < s->nprog_cols; ++i) sa.a.val_col[i] = (const uint64_t *)s->prog_col[i];
  for (size_t i = 0; i < js.consts.size(); ++i) sa.a.kc[i] = js.consts[i];
  sa.out = out_rows;
  sa.ticket = (uint32_t *)base;
  sa.out_n = (unsigned long long *)(base + 8);
  sa.status = (uint64_t *)(base + 16);
  sa.ntiles = (uint32_t)ntiles;
  NUT_HIP(hipMemsetAsync(base, 0, state, c->stream));
  size_t asz = sizeof sa;
  void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &sa, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz, HIP_LAUNCH_PARAM_END};
  c->timer.begin(c->stream, NUT_KERNEL_FILTER);
  // persistent workgroups (tiles by ticket): enough for full occupancy, never more than tiles
  const uint64_t per_cu = c->opt[NUT_OPT_SEL_BLOCKS] ? (uint64_t)c->opt[NUT_OPT_SEL_BLOCKS] : 8;
  const unsigned grid = (unsigned)std::min<uint64_t>(ntiles, (uint64_t)c->num_cus * per_cu);
  hipError_t e = hipModuleLaunchKernel(fn, grid, 1, 1, SEL_THREADS, 1, 1, 0, c->stream, nullptr, cfg);
  c->timer.end(c->stream);
  if (e != hipSuccess) return hip_fail(e, "hipModuleLaunchKernel (select kernel)");
  NUT_HIP(hipMemcpyAsync(c->host_pinned, base, 16, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  const uint32_t err = (uint32_t)(c->host_pinned[0] >> 32);
  if (err & 2u) return fail(NUT_ERR_INVALID_ARG, "nut_select_rows: division by zero in an expression");
  if (err & 1u) return fail(NUT_ERR_TIMEOUT, "nut_select_rows: look-back spin limit hit");
  *count_host = c->host_pinned[1];
  return NUT_OK;
}

// Computed projections (select_kernel.hpp eval_kernel): out[a][i] = program s->agg_val[a]
// at row rows[i] (rows NULL: i), valid[a][i] = its mask s->agg_mask[a] (1 without one).
static nut_status eval_prepare(const nut_agg_spec *s, JitShape &js) {
  if (!s->prog_mode) return fail(NUT_ERR_INVALID_ARG, "nut_eval_rows: needs an expression-mode spec (prog_mode = 1)");
  if (s->naggs < 1 || s->naggs > NUT_MAX_AGGS) return fail(NUT_ERR_INVALID_ARG, "nut_eval_rows: naggs not in [1, 8]");
  if (s->nprog_cols < 0 || s->nprog_cols > NUT_MAX_PROG_COLS)
    return fail(NUT_ERR_INVALID_ARG, "nut_eval_rows: bad program column count");
  nut_agg_spec q = *s;  // the value / mask programs alone
  q.where.n = 0;
  q.nkeys = 0;
  for (int a = 0; a < q.naggs; ++a) {
    if (!q.agg_val[a].n) return fail(NUT_ERR_INVALID_ARG, "nut_eval_rows: empty value program");
    q.agg_op[a] = NUT_AGG_SUM;
  }
  int32_t kinds[NUT_MAX_AGGS] = {};
  nut_status st = jit_shape(&q, kinds, js);
  if (st) return st;
  if (js.consts.size() > (size_t)kMaxConst)
    return fail(NUT_ERR_UNSUPPORTED, "nut_eval_rows: more than 64 distinct expression constants");
  return NUT_OK;
}

nut_status nut_eval_rows(nut_ctx *c, const nut_agg_spec *s, const int64_t *rows, uint64_t m, uint64_t *const *out,
                         uint8_t *const *valid) {
  if (!c || !s || (m && !out)) return fail(NUT_ERR_INVALID_ARG, "nut_eval_rows: NULL argument");
  JitShape js;
  nut_status st = eval_prepare(s, js);
  if (st || m == 0) return st;
  if (!rows && m > s->n) return fail(NUT_ERR_INVALID_ARG, "nut_eval_rows: m > s->n without row ids");
  for (int i = 0; i < s->nprog_cols; ++i)
    if (!s->prog_col[i]) return fail(NUT_ERR_INVALID_ARG, "nut_eval_rows: NULL program column");
  for (int a = 0; a < s->naggs; ++a)
    if (!out[a]) return fail(NUT_ERR_INVALID_ARG, "nut_eval_rows: NULL output column");
  DeviceGuard dg(c->device);
  hipFunction_t fn;
  st = jit_kernel(jit_eval_unit(js.src, sizeof(EvalArgs)), true, &fn);
  if (st) return st;
  st = c->misc.reserve(64);
  if (st) return st;
  uint32_t *derr = (uint32_t *)c->misc.ptr;
  EvalArgs ea;
  memset(&ea, 0, sizeof ea);
  ea.a.n = s->n;
  ea.a.nvals = s->nprog_cols;
  for (int i = 0; i < s->nprog_cols; ++i) ea.a.val_col[i] = (const uint64_t *)s->prog_col[i];
  for (size_t i = 0; i < js.consts.size(); ++i) ea.a.kc[i] = js.consts[i];
  ea.rows = rows;
  ea.m = m;
  for (int a = 0; a < s->naggs; ++a) {
    ea.out[a] = out[a];
    ea.valid[a] = valid ? valid[a] : nullptr;
  }
  ea.err = derr;
  ea.nout = s->naggs;
  NUT_HIP(hipMemsetAsync(derr, 0, 4, c->stream));
  size_t asz = sizeof ea;
  void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &ea, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz, HIP_LAUNCH_PARAM_END};
  const unsigned grid = (unsigned)std::min<uint64_t>((m + EV_THREADS - 1) / EV_THREADS, (uint64_t)c->num_cus * 16);
  c->timer.begin(c->stream, NUT_KERNEL_FILTER);
  hipError_t e = hipModuleLaunchKernel(fn, grid, 1, 1, EV_THREADS, 1, 1, 0, c->stream, nullptr, cfg);
  c->timer.end(c->stream);
  if (e != hipSuccess) return hip_fail(e, "hipModuleLaunchKernel (eval kernel)");
  NUT_HIP(hipMemcpyAsync(c->host_pinned, derr, 4, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  if ((uint32_t)c->host_pinned[0] & 2u) return fail(NUT_ERR_INVALID_ARG, "nut_eval_rows: division by zero in an expression");
  return NUT_OK;
}

nut_status nut_eval_jit_compile(const nut_agg_spec *s) {
  if (!s) return fail(NUT_ERR_INVALID_ARG, "nut_eval_jit_compile: NULL argument");
  JitShape js;
  nut_status st = eval_prepare(s, js);
  if (st) return st;
  return jit_kernel(jit_eval_unit(js.src, sizeof(EvalArgs)), false, nullptr);
}

// compile (no GPU needed) the scan kernel nut_select_rows would run for this spec
nut_status nut_select_jit_compile(const nut_agg_spec *s) {
  if (!s || !s->prog_mode) return fail(NUT_ERR_INVALID_ARG, "nut_select_jit_compile: needs an expression-mode spec");
  nut_agg_spec q = *s;
  q.naggs = 0;
  int32_t kinds[NUT_MAX_AGGS] = {};
  JitShape js;
  nut_status st = jit_shape(&q, kinds, js);
  if (st) return st;
  return jit_kernel(jit_select_unit(js.src, sizeof(SelArgs)), false, nullptr);
}

// The multi-GPU join's exchange step: one gp_level (gpart.hpp) over the keys with the row
// ids as payload, 256 digits of the owner hash's top byte, parts = digit ranges.
nut_status nut_hash_partition_i64(nut_ctx *c, const int64_t *keys, uint64_t n, int nparts, int64_t row0,
                                  int64_t *out_keys, int64_t *out_rows, uint64_t *counts_host) {
  if (!c || !counts_host || (n && (!keys || !out_keys || !out_rows)))
    return fail(NUT_ERR_INVALID_ARG, "nut_hash_partition_i64: NULL argument");
  if (nparts < 1 || nparts > GP_BINS) return fail(NUT_ERR_INVALID_ARG, "nut_hash_partition_i64: nparts not in [1, 256]");
  for (int p = 0; p < nparts; ++p) counts_host[p] = 0;
  if (n == 0) return NUT_OK;
  DeviceGuard dg(c->device);
  hipStream_t st = c->stream;
  int64_t *rows = nullptr;
  NUT_HIP(hipMallocAsync((void **)&rows, n * 8, st));
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, (uint64_t)c->num_cus * 16);
  hipLaunchKernelGGL(iota_kernel, dim3(g), dim3(256), 0, st, rows, n, row0);
  const uint64_t *src[GP_MAX_ARR] = {nullptr, (const uint64_t *)keys, nullptr, (const uint64_t *)rows};
  uint64_t *dst[GP_MAX_ARR] = {nullptr, (uint64_t *)out_keys, nullptr, (uint64_t *)out_rows};
  std::vector<GpSeg> segs{GpSeg{0, n, 0, 0}};
  std::vector<uint64_t> hist;
  GpMeta mm{c};
  nut_status e = gp_level(c, mm, segs, 56, src, dst, 4, false, false, hist);
  if (!e) {
    for (int d = 0; d < GP_BINS; ++d) counts_host[(d * nparts) >> 8] += hist[d];
    hipError_t he = hipStreamSynchronize(st);
    if (he != hipSuccess) e = hip_fail(he, "nut_hash_partition_i64");
  }
  (void)hipFreeAsync(rows, st);
  return e;
}

}  // extern "C"

namespace nut {
// The join's region build (join.hip): (key, row) records of `keys` partitioned by the top
// 16 bits of owner_hash(key ^ kx) — two gp_levels, 8 bits each — into outk / outr; tmpk /
// tmpr hold the first level.  counts[65536] = records per 16-bit partition, in order.
nut_status hash_partition16(nut_ctx *c, const int64_t *keys, uint64_t n, uint64_t kx, int64_t *tmpk, int64_t *tmpr,
                            int64_t *outk, int64_t *outr, std::vector<uint64_t> &counts, const int64_t *rows) {
  hipStream_t st = c->stream;
  counts.assign(65536, 0);
  if (n == 0) return NUT_OK;
  // row ids (`rows`, or indices staged in outr) partitioned into tmpr by level 1, into
  // outr by level 2
  if (!rows) {
    const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, (uint64_t)c->num_cus * 16);
    hipLaunchKernelGGL(iota_kernel, dim3(g), dim3(256), 0, st, outr, n, (int64_t)0);
    rows = outr;
  }
  const uint64_t *s1[GP_MAX_ARR] = {nullptr, (const uint64_t *)keys, nullptr, (const uint64_t *)rows};
  uint64_t *d1[GP_MAX_ARR] = {nullptr, (uint64_t *)tmpk, nullptr, (uint64_t *)tmpr};
  std::vector<GpSeg> segs{GpSeg{0, n, 0, 0}};
  std::vector<uint64_t> h1;
  GpMeta mm{c};
  nut_status e = gp_level(c, mm, segs, 56, s1, d1, 4, false, false, h1, nullptr, kx);
  if (e) return e;
  std::vector<GpSeg> s2;
  uint64_t run = 0;
  for (int d = 0; d < GP_BINS; ++d) {
    s2.push_back(GpSeg{run, h1[d], 0, 0});  // empty segments too: one histogram row per digit
    run += h1[d];
  }
  const uint64_t *src2[GP_MAX_ARR] = {nullptr, (const uint64_t *)tmpk, nullptr, (const uint64_t *)tmpr};
  uint64_t *d2[GP_MAX_ARR] = {nullptr, (uint64_t *)outk, nullptr, (uint64_t *)outr};
  std::vector<uint64_t> h2;
  e = gp_level(c, mm, s2, 48, src2, d2, 4, false, false, h2, nullptr, kx);
  if (e) return e;
  for (size_t i = 0; i < 65536; ++i) counts[i] = h2[i];
  return NUT_OK;
}
// ------------------------------------------------------------ multi-GPU merge (dist.cpp)
int groups_width(const nut_groups *g) { return g->nk + g->naggs; }

void groups_merge_spec(const nut_groups *g, const uint64_t *seg, uint64_t c, nut_agg_spec *s, nut_prog_node *nodes) {
  memset(s, 0, sizeof(*s));
  s->n = c;
  s->nkeys = g->nk;
  for (int j = 0; j < g->nk; ++j) s->keys[j] = (const int64_t *)(seg + (uint64_t)j * c);
  s->naggs = g->naggs;
  const bool prog = g->naggs > NUT_MAX_VALS;  // more partial columns than fused value slots
  if (prog) {
    s->prog_mode = 1;
    s->nprog_cols = g->naggs;
  } else {
    s->nvals = g->naggs;
  }
  for (int a = 0; a < g->naggs; ++a) {
    const int k = g->kinds[a];
    const bool f64 = k == AK_SUM_F64 || k == AK_MIN_F64 || k == AK_MAX_F64;
    const void *col = seg + (uint64_t)(g->nk + a) * c;
    // a COUNT partial is an int64 word: the merge adds them
    s->agg_op[a] = (k == AK_MIN_F64 || k == AK_MIN_I64) ? NUT_AGG_MIN
                   : (k == AK_MAX_F64 || k == AK_MAX_I64) ? NUT_AGG_MAX : NUT_AGG_SUM;
    if (prog) {
      s->prog_col[a] = col;
      s->prog_col_type[a] = f64 ? NUT_T_F64 : NUT_T_I64;
      nodes[a] = nut_prog_node{NUT_P_COL, a, 0};
      s->agg_val[a] = nut_prog{1, &nodes[a]};
    } else {
      s->val_col[a] = col;
      s->val_type[a] = f64 ? NUT_T_F64 : NUT_T_I64;
      s->agg_expr[a] = NUT_EX_COL;
      s->agg_arg[a][0] = a;
    }
  }
}

}  // namespace nut

extern "C" {

nut_status nut_groups_to_host(nut_groups *g, int64_t *keys, uint64_t *aggs, uint64_t cap) {
  if (!g) return fail(NUT_ERR_INVALID_ARG, "nut_groups_to_host: NULL argument");
  uint64_t n;
  nut_status st = nut_groups_size(g, &n);
  if (st) return st;
  if (n > cap)
    return fail(NUT_ERR_CAPACITY, "nut_groups_to_host: capacity " + std::to_string(cap) + " < " +
                                      std::to_string(n) + " groups");
  if (n == 0) return NUT_OK;
  if (!keys || (g->naggs && !aggs)) return fail(NUT_ERR_INVALID_ARG, "nut_groups_to_host: NULL output");
  nut_ctx *c = g->ctx;
  DeviceGuard dg(c->device);
  const int w = g->nk + g->naggs;
  uint64_t *dev = nullptr;
  NUT_HIP(hipMallocAsync((void **)&dev, (size_t)w * n * 8, c->stream));
  st = nut_groups_to_device(g, dev, n);
  if (st) {
    (void)hipFreeAsync(dev, c->stream);
    return st;
  }
  if (g->nk == 1 && n >= (1u << 16)) {
    // large one-key results are ordered on the device: sort the (unique) keys, then every
    // group finds its rank by binary search and is placed there
    const uint64_t saved_bytes = c->sort_bytes;
    const uint32_t saved_levels = c->sort_levels;
    uint64_t *buf = nullptr;
    const size_t nb = (size_t)n * 8;
    NUT_HIP(hipMallocAsync((void **)&buf, nb * (2 + (size_t)g->naggs), c->stream));
    int64_t *sorted = (int64_t *)buf, *dk = (int64_t *)(buf + n);
    uint64_t *da = buf + 2 * n;
    st = msd_sort_i64(c, (const int64_t *)dev, sorted, n, 0x8000000000000000ull);
    c->sort_bytes = saved_bytes;
    c->sort_levels = saved_levels;
    uint64_t *bstart = nullptr;
    if (!st) {
      const hipError_t he = hipMallocAsync((void **)&bstart, ((1ull << PL_BITS) + 2) * 8, c->stream);
      if (he != hipSuccess) st = hip_fail(he, "nut_groups_to_host (bucket index)");
    }
    if (!st) {
      const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, (uint64_t)c->num_cus * 16);
      hipLaunchKernelGGL(place_index_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, (const int64_t *)sorted, n,
                         bstart);
      hipLaunchKernelGGL(groups_place_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, (const uint64_t *)dev,
                         (const int64_t *)sorted, n, g->naggs, dk, da, (const uint64_t *)bstart);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) st = hip_fail(e, "nut_groups_to_host (device order)");
      if (!st) st = copy_to_host(c, keys, dk, nb);
      if (!st && g->naggs) st = copy_to_host(c, aggs, da, nb * g->naggs);
    }
    if (bstart) (void)hipFreeAsync(bstart, c->stream);
    (void)hipFreeAsync(buf, c->stream);
    (void)hipFreeAsync(dev, c->stream);
    return st;
  }
  std::vector<uint64_t> h((size_t)w * n);
  {
    hipError_t e = hipMemcpyAsync(h.data(), dev, (size_t)w * n * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) st = hip_fail(e, "nut_groups_to_host copy");
  }
  (void)hipFreeAsync(dev, c->stream);
  if (st) return st;
  std::vector<uint64_t> order(n);
  for (uint64_t i = 0; i < n; ++i) order[i] = i;
  const int nk = g->nk;
  std::sort(order.begin(), order.end(), [&](uint64_t x, uint64_t y) {
    int64_t a0 = (int64_t)h[x], b0 = (int64_t)h[y];
    if (a0 != b0) return a0 < b0;
    if (nk == 2) return (int64_t)h[n + x] < (int64_t)h[n + y];
    return false;
  });
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t src = order[i];
    for (int j = 0; j < nk; ++j) keys[i * nk + j] = (int64_t)h[(size_t)j * n + src];
    for (int a = 0; a < g->naggs; ++a) aggs[i * g->naggs + a] = h[(size_t)(nk + a) * n + src];
  }
  return NUT_OK;
}

// Small results on the on-chip path (the table's slots <= kSmallTail): the aggregation,
// the table's control words, the compaction and ONE copy of both into page-locked staging
// are queued back to back and the host waits once (nut_groupby + nut_groups_to_host wait
// three times and copy through pageable memory).  The compaction writes columns of the
// table's slot count (an upper bound of the groups), so nothing waits for the group count.
// *done = false: the table overflowed (more groups than hinted) or the shape takes another
// path — the caller runs the general one.
constexpr uint64_t kSmallTail = 1ull << 16;
nut_status groupby_small_to_host(nut_ctx *c, const nut_agg_spec *s, uint64_t group_hint, int64_t *keys,
                                 uint64_t *aggs, uint64_t cap, uint64_t *n_out, bool *done) {
  *done = false;
  const int64_t gp = c->opt[NUT_OPT_GB_PARTITION];
  if (s->nkeys == 0 || !s->n) return NUT_OK;
  if (gp == 1 || (gp != 0 && group_hint >= kGpMinGroups && s->n >= 4 * group_hint)) return NUT_OK;
  const uint64_t tcap = table_cap_for(group_hint ? group_hint : 8192);
  if (tcap + 1 > kSmallTail) return NUT_OK;
  nut_groups *g = new nut_groups();
  struct Free {
    nut_groups *g;
    ~Free() { nut_groups_free(g); }
  } free_g{g};
  g->ctx = c;
  g->nk = s->nkeys;
  g->naggs = s->naggs;
  for (int a = 0; a < s->naggs; ++a) g->kinds[a] = kind_of(s, a);
  c->gb_path = NUT_GB_ONCHIP;
  c->gb_levels = c->gb_optimistic = 0;
  nut_status st = alloc_table(g, tcap);
  if (!st) st = probe_priv_shape(g, s, group_hint, tcap);
  if (!st) st = launch_agg(g, s, group_hint, g->kinds);
  if (st) return st;
  const int nk = g->nk, na = g->naggs, w = nk + na;
  const uint64_t stride = g->gt.cap + 1;
  for (auto &b : c->stage)
    if (!b) NUT_HIP(hipHostMalloc((void **)&b, kStageBytes, hipHostMallocDefault));
  if ((stride * w + 2) * 8 > kStageBytes) return NUT_OK;
  uint64_t *dev = nullptr;
  NUT_HIP(hipMallocAsync((void **)&dev, (size_t)stride * w * 8, c->stream));
  struct FreeDev {
    uint64_t *p;
    hipStream_t s;
    ~FreeDev() { (void)hipFreeAsync(p, s); }
  } free_dev{dev, c->stream};
  uint64_t *host = (uint64_t *)c->stage[0];
  hipLaunchKernelGGL(gtable_sum_kernel, dim3(1), dim3(256), 0, c->stream, (const GTable *)g->dev_gt);
  NUT_HIP(hipMemcpyAsync(host, g->gt.ctl, 16, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipMemsetAsync(g->dev_cursors, 0, 64 * 8, c->stream));
  const uint64_t blocks = std::min<uint64_t>((stride + GT_CHUNK - 1) / GT_CHUNK, (uint64_t)c->num_cus * 8);
  hipLaunchKernelGGL(gtable_compact_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, (const GTable *)g->dev_gt,
                     nk, dev, stride, g->dev_cursors, 1, (const uint64_t *)nullptr);
  NUT_HIP(hipGetLastError());
  NUT_HIP(hipMemcpyAsync(host + 2, dev, (size_t)stride * w * 8, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  uint32_t ctl[4];
  memcpy(ctl, host, 16);
  if (ctl[1] & 2u) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: division by zero in an expression");
  if (ctl[1] & 1u) return NUT_OK;  // more groups than the table admits: the general path regrows it
  const uint64_t n = (uint64_t)ctl[0] + (nk == 1 && ctl[2] ? 1 : 0);
  *done = true;
  *n_out = n;
  if (n > cap)
    return fail(NUT_ERR_CAPACITY, "nut_groupby_to_host: capacity " + std::to_string(cap) + " < " + std::to_string(n) +
                                      " groups");
  // key-tuple order, rows out of the column-major staging (columns of `stride` rows)
  const uint64_t *h = host + 2;
  std::vector<uint32_t> order(n);
  for (uint64_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
  std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
    const int64_t a0 = (int64_t)h[x], b0 = (int64_t)h[y];
    if (a0 != b0) return a0 < b0;
    return nk == 2 && (int64_t)h[stride + x] < (int64_t)h[stride + y];
  });
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t src = order[i];
    for (int j = 0; j < nk; ++j) keys[i * nk + j] = (int64_t)h[(size_t)j * stride + src];
    for (int a = 0; a < na; ++a) aggs[i * na + a] = h[(size_t)(nk + a) * stride + src];
  }
  return NUT_OK;
}

nut_status nut_groupby_to_host(nut_ctx *c, const nut_agg_spec *s, uint64_t group_hint, int64_t *keys, uint64_t *aggs,
                               uint64_t cap, uint64_t *n_out) {
  if (!c || !n_out) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_to_host: NULL argument");
  *n_out = 0;
  nut_status st = validate(s);
  if (st) return st;
  DeviceGuard dg(c->device);
  st = groupby_ordered(c, s, group_hint, keys, aggs, cap, n_out);
  if (st != NUT_ERR_UNSUPPORTED) return st;
  *n_out = 0;
  bool done = false;
  if (keys && (aggs || !s->naggs)) {
    st = groupby_small_to_host(c, s, group_hint, keys, aggs, cap, n_out, &done);
    if (st || done) return st;
  }
  nut_groups *g = nullptr;
  st = nut_groupby(c, s, group_hint, &g);
  if (st) return st;
  uint64_t n = 0;
  st = nut_groups_size(g, &n);
  if (!st) {
    *n_out = n;
    st = nut_groups_to_host(g, keys, aggs, cap);
  }
  nut_groups_free(g);
  return st;
}

void nut_groups_free(nut_groups *g) {
  if (!g) return;
  if (g->mem) pool_give(g->ctx, g->mem, g->mem_bytes);  // kept for the next table
  delete g;
}

nut_status nut_groupby_i64_f64(nut_ctx *c, const int64_t *key, const double *val, uint64_t n, uint32_t mask,
                               uint64_t group_hint, nut_groups **out) {
  nut_agg_spec s;
  memset(&s, 0, sizeof(s));
  s.n = n;
  s.nkeys = 1;
  s.keys[0] = key;
  s.nvals = 1;
  s.val_col[0] = val;
  s.val_type[0] = NUT_T_F64;
  const int ops[4] = {NUT_AGG_SUM, NUT_AGG_COUNT, NUT_AGG_MIN, NUT_AGG_MAX};
  for (int b = 0; b < 4; ++b)
    if (mask & (1u << b)) {
      s.agg_op[s.naggs] = ops[b];
      s.agg_expr[s.naggs] = NUT_EX_COL;
      ++s.naggs;
    }
  if (s.naggs == 0) return fail(NUT_ERR_INVALID_ARG, "nut_groupby_i64_f64: empty aggregate mask");
  return nut_groupby(c, &s, group_hint, out);
}

nut_status nut_q1(nut_ctx *c, const int64_t *shipdate, const int64_t *returnflag, const int64_t *linestatus,
                  const double *qty, const double *price, const double *disc, uint64_t n, int64_t date_k,
                  nut_groups **out) {
  nut_agg_spec s;
  memset(&s, 0, sizeof(s));
  s.n = n;
  s.nkeys = 2;
  s.keys[0] = returnflag;
  s.keys[1] = linestatus;
  s.npred = 1;
  s.pred_col[0] = shipdate;
  s.pred_type[0] = NUT_T_I64;
  s.pred_op[0] = NUT_LE;
  s.pred_i64[0] = date_k;
  s.nvals = 3;
  s.val_col[0] = qty;
  s.val_col[1] = price;
  s.val_col[2] = disc;
  s.val_type[0] = s.val_type[1] = s.val_type[2] = NUT_T_F64;
  s.naggs = 4;
  s.agg_op[0] = NUT_AGG_SUM;
  s.agg_expr[0] = NUT_EX_COL;
  s.agg_arg[0][0] = 0;
  s.agg_op[1] = NUT_AGG_SUM;
  s.agg_expr[1] = NUT_EX_COL;
  s.agg_arg[1][0] = 1;
  s.agg_op[2] = NUT_AGG_SUM;
  s.agg_expr[2] = NUT_EX_MUL_1M;
  s.agg_arg[2][0] = 1;
  s.agg_arg[2][1] = 2;
  s.agg_op[3] = NUT_AGG_COUNT;
  return nut_groupby(c, &s, 8, out);
}

}  // extern "C"
