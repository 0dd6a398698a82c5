// aggregate.hip — host side of the fused  WHERE -> GROUP BY -> SUM/COUNT/MIN/MAX
// executor (BASELINE configs 3, 4): table lifecycle, kernel dispatch and the
// nut_groupby* / nut_groups_* / nut_q1 entry points of include/nutexec.h.
// Device code: agg_kernel.hpp + agg_ops.hpp (streaming kernel), gtable.hpp (global table).
#include <string.h>

#include <algorithm>
#include <vector>

#include "agg_kernel.hpp"
#include "jit.hpp"

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
  if (s->n) {
    for (int k = 0; k < s->nkeys; ++k)
      if (!s->keys[k]) return fail(NUT_ERR_INVALID_ARG, "nut_groupby: NULL key column");
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
  size_t o_gt = carve(sizeof(GTable));
  size_t o_cur = carve(64 * 8);
  size_t o_seg = carve(128 * 8);
  if (!(g->mem && g->mem_bytes >= off)) {
    if (g->mem) (void)hipFree(g->mem);
    g->mem = nullptr;
    NUT_HIP(hipMalloc(&g->mem, off));
    g->mem_bytes = off;
  }
  char *b = (char *)g->mem;
  GTable &t = g->gt;
  t.slot = (uint64_t *)(b + o_slot);
  t.agg = (uint64_t *)(b + o_agg);
  t.ak1 = (int64_t *)(b + o_a1);
  t.ak2 = (int64_t *)(b + o_a2);
  t.ctl = (uint32_t *)(b + o_ctl);
  t.cap = cap;
  t.log2cap = ilog2(cap);
  t.limit = (uint32_t)std::min<uint64_t>(cap - cap / 4, 0xFFFFFFF0ull);
  t.arena_cap = (uint32_t)std::min<uint64_t>(arena, 0xFFFFFFF0ull);
  t.naggs = g->naggs;
  t.kinds = pack_kinds(g->kinds, g->naggs);
  g->dev_gt = (GTable *)(b + o_gt);
  g->dev_cursors = (unsigned long long *)(b + o_cur);
  g->dev_segbase = (uint64_t *)(b + o_seg);
  hipStream_t st = g->ctx->stream;
  NUT_HIP(hipMemsetAsync(t.ctl, 0, 64, st));
  NUT_HIP(hipMemcpyAsync(g->dev_gt, &g->gt, sizeof(GTable), hipMemcpyHostToDevice, st));
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)g->ctx->num_cus * 8);
  hipLaunchKernelGGL(gtable_init_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const GTable *)g->dev_gt, g->nk);
  NUT_HIP(hipGetLastError());
  return NUT_OK;
}

nut_status read_ctl(nut_groups *g, uint32_t *ctl4) {
  nut_ctx *c = g->ctx;
  NUT_HIP(hipMemcpyAsync(c->host_pinned, g->gt.ctl, 16, hipMemcpyDeviceToHost, c->stream));
  NUT_HIP(hipStreamSynchronize(c->stream));
  memcpy(ctl4, c->host_pinned, 16);
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
KernelFn pick_kernel(int nk, bool priv, int shape, bool vec) {
  if (!vec) shape = SHAPE_GENERIC;
  if (priv) {
    if (shape == SHAPE_Q1) return agg_kernel<2, true, kBdPriv, ShapeQ1, 1>;
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

// launch the streaming aggregation of spec's rows into g's table.  `kinds` are the
// per-row update kinds (COUNT partials are merged as integer sums).
nut_status launch_agg(nut_groups *g, const nut_agg_spec *s, uint64_t group_hint, const int32_t *kinds) {
  nut_ctx *c = g->ctx;
  if (s->n == 0) return NUT_OK;
  AggArgs a;
  memset(&a, 0, sizeof(a));
  a.n = s->n;
  // nkeys == 0 (global aggregate) runs the one-key kernels with every key = 0
  a.nokey = s->nkeys == 0 ? 1 : 0;
  a.keys[0] = (const uint64_t *)(s->nkeys ? s->keys[0] : nullptr);
  a.keys[1] = s->nkeys == 2 ? (const uint64_t *)s->keys[1] : a.keys[0];
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

  // on-chip table: 4x the expected groups (load <= 1/4: a key almost always sits in
  // its 4-slot home bucket) within the LDS budget
  const size_t lds_max = 160 * 1024;
  const int na = s->naggs;
  // (32 slots = 8 buckets x 32 B = one pass over the 64 LDS banks: for <= 8 groups two
  // home buckets never conflict — distinct buckets hit distinct banks, equal ones broadcast)
  uint64_t want = group_hint ? 4 * group_hint : 4096;
  uint32_t lcap = 32;
  while (lcap < want && lds_bytes(lcap * 2, g->nk, na, false, 0, kBdShared) <= lds_max) lcap *= 2;
  if (group_hint > 8ull * lcap) lcap = 0;  // hot keys cannot fit on chip: straight to HBM
  // private accumulators when every expected group fits P per thread, 2 blocks per CU
  int P = 0;
  if (lcap && group_hint && group_hint <= (uint64_t)kPrivMax && na > 0) {
    P = (int)group_hint;
    if (lds_bytes(lcap, g->nk, na, true, P, kBdPriv) > lds_max / 2) P = 0;
  }
  const bool priv = P > 0;
  const int bd = priv ? kBdPriv : kBdShared;
  a.lds_cap = lcap;
  a.lds_limit = lcap - lcap / 4;
  a.lds_log2 = lcap ? ilog2(lcap) : 0;
  a.priv = P;
  a.gt = g->dev_gt;
  const size_t lb = lds_bytes(lcap, g->nk, na, priv, P, bd);
  int blocks_per_cu = lb ? (int)std::max<size_t>(1, std::min<size_t>(bd == 512 ? 4 : 8, lds_max / lb)) : 4;
  uint64_t pairs = (s->n + 1) / 2;
  uint64_t blocks = std::min<uint64_t>((uint64_t)c->num_cus * blocks_per_cu, (pairs + bd - 1) / bd);
  if (blocks == 0) blocks = 1;
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
  const int shape = detect_shape(s, kinds, a);
  KernelFn fn = pick_kernel(g->nk, priv, shape, a.vec != 0);
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
  if (need <= g->gt.limit && (g->nk == 1 || (uint64_t)ctl[3] + extra <= g->gt.arena_cap)) return NUT_OK;
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
  g->dev_cursors = fresh.dev_cursors;
  g->dev_segbase = fresh.dev_segbase;
  fresh.mem = nullptr;
  return NUT_OK;
}

}  // namespace

extern "C" {

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
  for (int attempt = 0;; ++attempt) {
    st = alloc_table(g, cap);
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
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)c->num_cus * 8);
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
  uint64_t blocks = std::min<uint64_t>((stride + 255) / 256, (uint64_t)c->num_cus * 8);
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
  std::vector<uint64_t> h((size_t)w * n);
  if (!st) {
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

void nut_groups_free(nut_groups *g) {
  if (!g) return;
  if (g->mem) {
    DeviceGuard dg(g->ctx->device);
    (void)hipStreamSynchronize(g->ctx->stream);
    (void)hipFree(g->mem);
  }
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
