// sql_exec_scan.cpp — executing FILTER / SORT plans (scans with any WHERE, projections,
// ORDER BY / LIMIT over row ids) and binding plans to nut_agg_spec (build_spec).
#include "sql_plan.hpp"

namespace nut {
namespace plan {


Verdict resolve_i64(int op, const CVal &c, int &out_op, int64_t &k) {
  i128 v;
  bool frac = false;
  if (c.is_int)
    v = c.v;
  else
    v = dec_floor(c.dec, frac);
  out_op = op;
  if (frac) {  // x <cmp> v with floor(v) < v < floor(v)+1
    switch (op) {
      case NUT_LT:
      case NUT_LE: out_op = NUT_LE; break;
      case NUT_GT:
      case NUT_GE: out_op = NUT_GT; break;
      case NUT_EQ: return V_FALSE;
      default: return V_TRUE;
    }
  }
  if (v > INT64_MAX) return (out_op == NUT_LT || out_op == NUT_LE || out_op == NUT_NE) ? V_TRUE : V_FALSE;
  if (v < INT64_MIN) return (out_op == NUT_GT || out_op == NUT_GE || out_op == NUT_NE) ? V_TRUE : V_FALSE;
  k = (int64_t)v;
  return V_PRED;
}

double resolve_f64(const CVal &c) { return c.is_int ? (double)c.v : c.dec.to_f64(); }

const nut_column *bind(const nut_plan &p, int ci, const nut_column *cols, int ncols) {
  for (int i = 0; i < ncols; ++i)
    if (cols[i].name && ieq(cols[i].name, p.cols[ci])) return &cols[i];
  // a qualified name (a single-table plan's n1.n_name) binds to its bare column otherwise
  const size_t dot = p.cols[ci].find('.');
  if (dot != std::string::npos)
    for (int i = 0; i < ncols; ++i)
      if (cols[i].name && ieq(cols[i].name, sv(p.cols[ci]).substr(dot + 1))) return &cols[i];
  return nullptr;
}



bool needs_key_progs(const nut_plan &p) {
  if (!p.compiled || p.kind != NUT_PLAN_GROUPBY) return false;
  if (p.keys.size() > NUT_MAX_KEYS) return true;
  for (int k : p.keys)
    if (k < 0) return true;
  for (const PlanAgg &a : p.aggs)
    if (a.distinct) return true;
  return false;
}

// ORDER BY ... LIMIT: the positions (ascending) of the n keys that can reach the first
// `need` places (nut_topk_positions) in *pos, *m of them; *m = n (pos untouched) when a
// full sort is as cheap (few keys, a limit close to n, or the option off)
nut_status topk_reduce(nut_ctx *c, const nut_plan &p, const void *keys, int type, bool desc, uint64_t n, DevBuf &pos,
                       uint64_t *m) {
  *m = n;
  if (!p.has_limit || !c->opt[NUT_OPT_TOPK] || n < (1u << 16)) return NUT_OK;
  const uint64_t need = p.offset > n ? n : std::min<uint64_t>(n, p.offset + std::min<uint64_t>(p.limit, n));
  if (need == 0) {
    *m = 0;
    return NUT_OK;
  }
  if (need > n / 4) return NUT_OK;
  const uint64_t cap = n / 2;
  if (pos.alloc(c, cap * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (top-k)");
  uint64_t cnt = 0;
  nut_status s = nut_topk_positions(c, keys, type, desc ? 1 : 0, n, need, (int64_t *)pos.p, cap, &cnt);
  if (s == NUT_ERR_CAPACITY) return NUT_OK;  // heavy ties at the boundary: the full sort
  if (s) return s;
  *m = cnt;
  return NUT_OK;
}

bool computed_proj(const nut_plan &p, size_t j) { return j < p.proj_val.size() && !p.proj_val[j].empty(); }

// Row-id scans (expression mode): ORDER BY with projected columns / several keys, several
// projections, computed projections.  The selected row ids (nut_select_rows, ascending)
// are sorted by the ORDER BY keys — one stable (key, row id) sort per key, the least
// significant first (nut_sort_pairs); with a LIMIT only the rows top-k selection keeps on
// the most significant key are sorted, and without ORDER BY only the first offset + limit
// ids are kept.  Every plain projection is then gathered through the ids and every
// computed one evaluated at them (nut_eval_rows, up to 8 programs per launch); a computed
// projection's NULL mask fills the result's validity flags.
nut_status exec_sort_rows(nut_ctx *c, const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts,
                          uint64_t n, nut_result *r) {
  // (ORDER BY keys checked by scan_route: int64 or float64, no strings)
  const size_t np = p.projs.size();
  // computed projections: groups of <= NUT_MAX_AGGS programs, one eval spec each
  std::vector<size_t> comp;
  for (size_t j = 0; j < np; ++j)
    if (computed_proj(p, j)) comp.push_back(j);
  std::deque<ProgStore> stores;
  std::vector<nut_agg_spec> specs;
  std::vector<std::vector<size_t>> members;
  std::vector<int> ctype(np, NUT_T_I64);
  for (size_t g0 = 0; g0 < comp.size(); g0 += NUT_MAX_AGGS) {
    nut_plan q;
    q.compiled = true;
    q.cols = p.cols;
    members.emplace_back();
    for (size_t t = g0; t < comp.size() && t < g0 + NUT_MAX_AGGS; ++t) {
      PlanAgg a{};
      a.op = NUT_AGG_SUM;
      a.val = p.proj_val[comp[t]];
      a.mask = p.proj_mask[comp[t]];
      q.aggs.push_back(std::move(a));
      members.back().push_back(comp[t]);
    }
    specs.emplace_back();
    stores.emplace_back();
    std::vector<int> f64;
    nut_status s = build_spec(q, bound, dicts, n, specs.back(), stores.back(), f64);
    if (s) return s;
    for (size_t t = 0; t < members.back().size(); ++t) ctype[members.back()[t]] = f64[t] ? NUT_T_F64 : NUT_T_I64;
  }
  // a string output: a plain dictionary column, or a computed projection that is one (the
  // NULL-masked column of a LEFT-joined table)
  std::vector<int> sdict(np, -1);
  for (size_t j = 0; j < np; ++j) {
    int dc = p.projs[j];
    if (computed_proj(p, j))
      dc = p.proj_val[j].size() == 1 && (p.proj_val[j][0].op == NUT_P_COL || p.proj_val[j][0].op == P_SUBSTR)
               ? p.proj_val[j][0].col
               : -1;
    if (dc >= 0 && dicts && dicts[dc]) sdict[j] = dc;
    r->names.push_back(p.outs[j].name);
    r->types.push_back(sdict[j] >= 0 ? NUT_T_STR : p.projs[j] >= 0 ? bound[p.projs[j]]->type : ctype[j]);
  }
  uint64_t cnt = 0;
  DevBuf rows, perm, keys;
  if (!p.never && n) {
    nut_agg_spec sp;
    ProgStore store;
    std::vector<int> agg_f64;
    nut_plan q = p;  // the WHERE program alone
    q.aggs.clear();
    nut_status s = build_spec(q, bound, dicts, n, sp, store, agg_f64);
    if (s) return s;
    NUT_HIP(rows.alloc(c, n * 8));
    s = nut_select_rows(c, &sp, (int64_t *)rows.p, &cnt);
    if (s) return s;
  }
  if (cnt && p.has_limit && p.sort_keys.empty()) {
    // no ORDER BY: the first offset + limit selected rows (table order)
    const uint64_t need = p.offset >= cnt ? 0 : p.offset + std::min<uint64_t>(p.limit, cnt - p.offset);
    cnt = std::min(cnt, need);
  } else if (cnt && p.has_limit) {
    // top-k on the most significant key: keep the candidate rows (ascending ids)
    const nut_column *kc = bound[p.sort_keys[0].first];
    NUT_HIP(keys.alloc(c, cnt * 8));
    nut_status s = nut_gather_u64(c, (const uint64_t *)kc->data, (const int64_t *)rows.p, cnt, 0, (uint64_t *)keys.p);
    DevBuf pos;
    uint64_t m2 = cnt;
    if (!s) s = topk_reduce(c, p, keys.p, kc->type, p.sort_keys[0].second, cnt, pos, &m2);
    if (s) return s;
    if (m2 < cnt) {
      NUT_HIP(perm.alloc(c, std::max<uint64_t>(m2, 1) * 8));
      s = nut_gather_u64(c, (const uint64_t *)rows.p, (const int64_t *)pos.p, m2, 0, (uint64_t *)perm.p);
      if (s) return s;
      std::swap(rows.p, perm.p);
      cnt = m2;
      perm.reset();  // (stream-ordered free of the full id list)
    }
    keys.reset();
  }
  const uint64_t m = std::max<uint64_t>(cnt, 1);
  NUT_HIP(hipMalloc(&r->dev, m * 8 * np));
  r->dev_stride = cnt;
  int nvalid = 0;
  r->valid_of.assign(np, -1);
  for (size_t j : comp)
    if (!p.proj_mask[j].empty()) r->valid_of[j] = nvalid++;
  if (nvalid) NUT_HIP(hipMalloc(&r->valid, m * nvalid));
  if (cnt) {
    NUT_HIP(perm.alloc(c, m * 8));
    NUT_HIP(keys.alloc(c, m * 8));
    nut_status s = NUT_OK;
    for (size_t i = p.sort_keys.size(); i-- > 0 && !s;) {
      const nut_column *kc = bound[p.sort_keys[i].first];
      s = nut_gather_u64(c, (const uint64_t *)kc->data, (const int64_t *)rows.p, cnt, 0, (uint64_t *)keys.p);
      if (!s) s = nut_sort_pairs(c, keys.p, kc->type, p.sort_keys[i].second ? 1 : 0, (const int64_t *)rows.p,
                                 (int64_t *)perm.p, cnt);
      std::swap(rows.p, perm.p);  // the sorted row ids feed the next (more significant) key
    }
    for (size_t j = 0; j < np && !s; ++j)
      if (!computed_proj(p, j))
        s = nut_gather_u64(c, (const uint64_t *)bound[p.projs[j]]->data, (const int64_t *)rows.p, cnt, 0,
                           (uint64_t *)r->dev + j * cnt);
    for (size_t g = 0; g < specs.size() && !s; ++g) {
      uint64_t *outs[NUT_MAX_AGGS] = {};
      uint8_t *vals[NUT_MAX_AGGS] = {};
      for (size_t t = 0; t < members[g].size(); ++t) {
        const size_t j = members[g][t];
        outs[t] = (uint64_t *)r->dev + j * cnt;
        vals[t] = r->valid_of[j] >= 0 ? r->valid + (uint64_t)r->valid_of[j] * cnt : nullptr;
      }
      s = nut_eval_rows(c, &specs[g], (const int64_t *)rows.p, cnt, outs, vals);
    }
    if (!s) s = nut_ctx_sync(c);
    if (s) return s;
  }
  const uint64_t off = p.has_limit ? std::min(p.offset, cnt) : 0;
  uint64_t nrows = cnt - off;
  if (p.has_limit) nrows = std::min(nrows, p.limit);
  r->dev_off = off;
  r->nrows = nrows;
  for (size_t j = 0; j < np; ++j) {  // decode string columns (codes -> text; NULL rows: empty)
    if (r->types[j] != NUT_T_STR) continue;
    r->strs.resize(np);
    std::vector<int64_t> codes(nrows);
    std::vector<uint8_t> ok(nrows, 1);
    if (nrows) NUT_HIP(hipMemcpy(codes.data(), (const int64_t *)r->dev + j * r->dev_stride + off, nrows * 8,
                                 hipMemcpyDeviceToHost));
    if (nrows && r->valid_of[j] >= 0)
      NUT_HIP(hipMemcpy(ok.data(), r->valid + (uint64_t)r->valid_of[j] * r->dev_stride + off, nrows,
                        hipMemcpyDeviceToHost));
    const Dict *d = dicts[sdict[j]];
    r->strs[j].reserve(nrows);
    for (uint64_t i = 0; i < nrows; ++i) {
      const std::string *v = ok[i] ? d->decode(codes[i]) : nullptr;
      r->strs[j].push_back(v ? *v : std::string());
    }
  }
  return NUT_OK;
}

// Which executor a FILTER / SORT plan takes over its bound columns (host only; also the
// nut_plan_route test hook).  Fused scans compare and sort int64 words: a float64 column
// (projected or compared) reruns in expression mode, where the WHERE is a program that
// compares in f64 and a single-key sort maps the f64 bits to int64 words in the IEEE
// total order first (S_EXPR_SORT_F64); string FILTER scans rerun the same way (codes
// gathered, then decoded).  Several keys / projections and computed projections are
// row-id scans (exec_sort_rows: nut_sort_pairs sorts f64 keys in the same total order).
nut_status scan_route(const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts, ScanRoute *route) {
  bool computed = false;
  for (size_t j = 0; j < p.projs.size(); ++j) computed = computed || computed_proj(p, j);
  if (computed || (p.kind == NUT_PLAN_SORT &&
                   !(p.sort_keys.size() == 1 && p.projs.size() == 1 && p.sort_keys[0].first == p.proj))) {
    for (const auto &k : p.sort_keys) {
      if (dicts && dicts[k.first])
        return fail(NUT_ERR_PLAN, "ORDER BY string column '" + p.cols[k.first] + "' is not executed (dictionary codes "
                                  "are in first-seen order)");
      if (bound[k.first]->type != NUT_T_I64 && bound[k.first]->type != NUT_T_F64)
        return fail(NUT_ERR_PLAN, "ORDER BY column '" + p.cols[k.first] + "' must be int64 or float64");
    }
    *route = S_ROWID;
    return NUT_OK;
  }
  bool f64 = false;
  for (int pj : p.projs) f64 = f64 || bound[pj]->type == NUT_T_F64;
  for (const PlanPred &pr : p.preds) f64 = f64 || bound[pr.col]->type == NUT_T_F64;
  if (!p.compiled && (f64 || (p.kind == NUT_PLAN_FILTER && dicts && dicts[p.proj]))) {
    *route = S_RERUN_EXPR;
    return NUT_OK;
  }
  for (int pj : p.projs)
    if (dicts && dicts[pj] && !(p.compiled && p.kind == NUT_PLAN_FILTER))
      return fail(NUT_ERR_PLAN, "column '" + p.cols[pj] + "' holds strings: sorts and single-column fused scans of "
                                "strings are not executed");
  for (const PlanPred &pr : p.preds)
    if (pr.c.is_str) return fail(NUT_ERR_PLAN, "string constant " + cval_str(pr.c) + " compared with an int64 column");
  for (int pj : p.projs)
    if (bound[pj]->type != NUT_T_I64 && !(p.compiled && bound[pj]->type == NUT_T_F64))
      return fail(NUT_ERR_PLAN, "column '" + p.cols[pj] + "' must be int64 or float64 for this scan/sort");
  if (p.compiled)
    *route = p.kind == NUT_PLAN_FILTER ? S_EXPR_FILTER : f64 ? S_EXPR_SORT_F64 : S_EXPR_SORT;
  else
    *route = p.kind == NUT_PLAN_FILTER ? S_FUSED_FILTER : S_FUSED_SORT;
  return NUT_OK;
}

const char *scan_route_name(ScanRoute r) {
  static const char *const k[] = {"rowid-scan", "rerun-expression", "expr-filter", "expr-sort", "expr-sort-f64-order",
                                  "fused-filter", "fused-sort"};
  return k[r];
}

nut_status exec_scan(nut_ctx *c, const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts,
                     uint64_t n, nut_result *r) {
  ScanRoute route;
  nut_status rs = scan_route(p, bound, dicts, &route);
  if (rs) return rs;
  if (route == S_ROWID) return exec_sort_rows(c, p, bound, dicts, n, r);
  if (route == S_RERUN_EXPR) {  // the WHERE as one program, then the expression-mode scan
    nut_plan q = p;
    std::vector<PProg> cs;
    for (const PlanPred &pr : p.preds) cs.push_back(pred_prog(pr));
    q.compiled = true;
    q.preds.clear();
    q.where = and_all(cs);
    return exec_scan(c, q, bound, dicts, n, r);
  }
  const nut_column *col = bound[p.proj];
  for (size_t j = 0; j < p.projs.size(); ++j) {
    r->names.push_back(p.outs[j].name);
    r->types.push_back(dicts && dicts[p.projs[j]] ? NUT_T_STR : bound[p.projs[j]]->type);
  }
  int op = NUT_GE;
  int64_t k = INT64_MIN;  // no predicate: every row passes
  bool none = p.never || n == 0;
  if (!p.compiled && !none && !p.preds.empty()) {
    Verdict v = resolve_i64(p.preds[0].op, p.preds[0].c, op, k);
    if (v == V_FALSE) none = true;
    if (v == V_TRUE) {
      op = NUT_GE;
      k = INT64_MIN;
    }
  }
  uint64_t cnt = 0;
  if (!none && p.compiled) {
    // expression-mode scan: row ids where the WHERE program holds, then the projected
    // column gathered through them (ascending ids), then sorted for ORDER BY
    nut_agg_spec sp;
    ProgStore store;
    std::vector<int> agg_f64;
    nut_status s = build_spec(p, bound, dicts, n, sp, store, agg_f64);
    if (s) return s;
    DevBuf rows;
    NUT_HIP(rows.alloc(c, n * 8));
    s = nut_select_rows(c, &sp, (int64_t *)rows.p, &cnt);
    if (s) return s;
    const size_t k = p.kind == NUT_PLAN_FILTER ? p.projs.size() : 1;
    NUT_HIP(hipMalloc(&r->dev, std::max<uint64_t>(cnt, 1) * 8 * k));
    if (p.kind == NUT_PLAN_FILTER) {
      r->dev_stride = cnt;
      for (size_t j = 0; j < k && !s; ++j)
        s = nut_gather_u64(c, (const uint64_t *)bound[p.projs[j]]->data, (const int64_t *)rows.p, cnt, 0,
                           (uint64_t *)r->dev + j * cnt);
    } else {
      DevBuf vals, pos, cv;
      NUT_HIP(vals.alloc(c, std::max<uint64_t>(cnt, 1) * 8));
      s = nut_gather_u64(c, (const uint64_t *)col->data, (const int64_t *)rows.p, cnt, 0, (uint64_t *)vals.p);
      // float64: the words sort (and top-k select) as int64 in the IEEE total order, and
      // map back after the sort (-0.0 before +0.0, NaNs at the ends by sign)
      const bool fo = route == S_EXPR_SORT_F64;
      if (!s && fo) s = f64_signed_order(c, (const uint64_t *)vals.p, (uint64_t *)vals.p, cnt);
      uint64_t m2 = cnt;  // ORDER BY ... LIMIT: only the top-k candidates are sorted
      if (!s) s = topk_reduce(c, p, vals.p, NUT_T_I64, p.desc, cnt, pos, &m2);
      if (!s && m2 < cnt) {
        if (cv.alloc(c, std::max<uint64_t>(m2, 1) * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (top-k)");
        s = nut_gather_u64(c, (const uint64_t *)vals.p, (const int64_t *)pos.p, m2, 0, (uint64_t *)cv.p);
        std::swap(vals.p, cv.p);
        cnt = m2;
      }
      if (!s) s = p.desc ? nut_sort_i64_desc(c, (const int64_t *)vals.p, (int64_t *)r->dev, cnt)
                         : nut_sort_i64(c, (const int64_t *)vals.p, (int64_t *)r->dev, cnt);
      if (!s && fo) s = f64_signed_order(c, (const uint64_t *)r->dev, (uint64_t *)r->dev, cnt);
    }
    if (!s) s = nut_ctx_sync(c);
    if (s) return s;
  } else if (!none) {
    NUT_HIP(hipMalloc(&r->dev, n * 8));
    if (p.kind == NUT_PLAN_FILTER) {
      nut_status s = nut_filter_i64(c, (const int64_t *)col->data, n, op, k, (int64_t *)r->dev, &cnt);
      if (s) return s;
    } else {
      const int64_t *src = (const int64_t *)col->data;
      DevBuf tmp;
      cnt = n;
      if (!p.preds.empty() && !(op == NUT_GE && k == INT64_MIN)) {
        NUT_HIP(tmp.alloc(c, n * 8));
        nut_status s = nut_filter_i64(c, src, n, op, k, (int64_t *)tmp.p, &cnt);
        if (s) return s;
        src = (const int64_t *)tmp.p;
      }
      DevBuf pos, cv;
      uint64_t m2 = cnt;  // ORDER BY ... LIMIT: only the top-k candidates are sorted
      nut_status s = topk_reduce(c, p, src, NUT_T_I64, p.desc, cnt, pos, &m2);
      if (s) return s;
      if (m2 < cnt) {
        if (cv.alloc(c, std::max<uint64_t>(m2, 1) * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (top-k)");
        s = nut_gather_u64(c, (const uint64_t *)src, (const int64_t *)pos.p, m2, 0, (uint64_t *)cv.p);
        if (s) return s;
        src = (const int64_t *)cv.p;
        cnt = m2;
      }
      s = p.desc ? nut_sort_i64_desc(c, src, (int64_t *)r->dev, cnt) : nut_sort_i64(c, src, (int64_t *)r->dev, cnt);
      if (s) return s;
      s = nut_ctx_sync(c);
      if (s) return s;
    }
  }
  uint64_t off = p.has_limit ? std::min(p.offset, cnt) : 0;
  uint64_t rows = cnt - off;
  if (p.has_limit) rows = std::min(rows, p.limit);
  r->dev_off = off;
  r->nrows = rows;
  for (size_t j = 0; j < p.projs.size(); ++j) {  // decode string columns (codes -> text)
    if (r->types[j] != NUT_T_STR) continue;
    r->strs.resize(p.projs.size());
    std::vector<int64_t> codes(rows);
    if (rows) NUT_HIP(hipMemcpy(codes.data(), (const int64_t *)r->dev + j * r->dev_stride + off, rows * 8,
                                hipMemcpyDeviceToHost));
    const Dict *d = dicts[p.projs[j]];
    r->strs[j].reserve(rows);
    for (int64_t cde : codes) {
      const std::string *v = d->decode(cde);
      r->strs[j].push_back(v ? *v : std::string());
    }
  }
  return NUT_OK;
}

HVal having_val(const HNode &h, const std::vector<std::vector<uint64_t>> &cols, const std::vector<int> &types,
                uint64_t g) {
  if (h.k == H_CONST) return HVal{h.is_int, h.i, h.f};
  const uint64_t w = cols[h.out][g];
  if (types[h.out] == NUT_T_I64) return HVal{true, (int64_t)w, 0.0};
  double f;
  memcpy(&f, &w, 8);
  return HVal{false, 0, f};
}
bool having_true(const HNode &h, const std::vector<std::vector<uint64_t>> &cols, const std::vector<int> &types,
                 uint64_t g) {
  switch (h.k) {
    case H_BOOL: return h.b;
    case H_NOT: return !having_true(h.kids[0], cols, types, g);
    case H_AND: return having_true(h.kids[0], cols, types, g) && having_true(h.kids[1], cols, types, g);
    case H_OR: return having_true(h.kids[0], cols, types, g) || having_true(h.kids[1], cols, types, g);
    case H_CMP: {
      const HVal a = having_val(h.kids[0], cols, types, g), b = having_val(h.kids[1], cols, types, g);
      int c;
      if (a.is_int && b.is_int) {
        c = a.i < b.i ? -1 : a.i > b.i ? 1 : 0;
      } else {
        const double x = a.is_int ? (double)a.i : a.f, y = b.is_int ? (double)b.i : b.f;
        if (x != x || y != y) return h.op == NUT_NE;  // NaN compares unequal
        c = x < y ? -1 : x > y ? 1 : 0;
      }
      switch (h.op) {
        case NUT_LT: return c < 0;
        case NUT_LE: return c <= 0;
        case NUT_GT: return c > 0;
        case NUT_GE: return c >= 0;
        case NUT_EQ: return c == 0;
        default: return c != 0;
      }
    }
    default: return false;
  }
}

// the nut_agg_spec of an aggregate plan over bound columns (program nodes live in store)
// String programs: a dictionary column or string constant may only meet another string
// in = / != (IN and CASE x WHEN lower to those), or be a GROUP BY key.
// Each table has its own dictionary: two columns compare only when their codes come from
// the same one (columns of one table; a join's two tables do not).
nut_status check_strings(const nut_plan &p, const PProg &pp, const Dict *const *dicts, const char *what) {
  static const Dict *const kConst = reinterpret_cast<const Dict *>(uintptr_t(1));  // a string constant
  std::vector<const Dict *> st;
  for (const PNode &n : pp) {
    const int op = n.op;
    const int k = pnode_arity(op);
    const Dict *a[3] = {nullptr, nullptr, nullptr};
    for (int i = k - 1; i >= 0; --i) {
      if (st.empty()) return NUT_OK;  // malformed: nut_prog_type reports it
      a[i] = st.back();
      st.pop_back();
    }
    if (op == NUT_P_COL || op == P_SUBSTR) {  // (a substring: a code of its column's dictionary)
      st.push_back(dicts[n.col]);
      continue;
    }
    if (op == NUT_P_I64 || op == NUT_P_F64) {
      st.push_back(n.c.is_str ? kConst : nullptr);
      continue;
    }
    if ((op == NUT_P_EQ || op == NUT_P_NE) && (a[0] != nullptr) != (a[1] != nullptr))
      return fail(NUT_ERR_PLAN, std::string(what) + ": a string compared with a number");
    if ((op == NUT_P_EQ || op == NUT_P_NE) && a[0] && a[1] && a[0] != kConst && a[1] != kConst && a[0] != a[1])
      return fail(NUT_ERR_PLAN, std::string(what) + ": string columns of two tables compared (their dictionaries "
                                                    "differ; only columns of one table compare)");
    if (!(op == NUT_P_EQ || op == NUT_P_NE) && (a[0] || a[1] || a[2]))
      return fail(NUT_ERR_PLAN, std::string(what) + ": strings are executed in = / != / IN and as GROUP BY keys only");
    st.push_back(nullptr);
  }
  if (!st.empty() && st.back()) return fail(NUT_ERR_PLAN, std::string(what) + ": a string value (only count() takes strings)");
  return NUT_OK;
}

int key_dict_col(const nut_plan &p, size_t j) {
  if (j < p.keys.size() && p.keys[j] >= 0) return p.keys[j];
  if (j < p.key_progs.size() && p.key_progs[j].size() == 1 && p.key_progs[j][0].op == P_SUBSTR)
    return p.key_progs[j][0].col;
  return -1;
}

// substring(s, off, len), bytes (ClickHouse `substring`): the window starts at byte off - 1
// (off >= 1) or |off| bytes before the end (off < 0), is len bytes long (len < 0: ends |len|
// bytes before the end; no len, kHuge: at the end), and is clipped to the string — a window
// starting before the string keeps only its part inside; off = 0 gives ''
std::string substr_bytes(const std::string &s, int off, i128 len) {
  const i128 sz = (i128)s.size();
  if (off == 0) return std::string();
  const i128 w0 = off > 0 ? (i128)off - 1 : sz + off;
  const i128 w1 = len >= kHuge ? sz : len >= 0 ? w0 + len : sz + len;
  const i128 b = std::max<i128>(0, std::min(w0, sz)), e = std::min(w1, sz);
  return e > b ? s.substr((size_t)b, (size_t)(e - b)) : std::string();
}

namespace {
// substring(col, off, len) over a dictionary (P_SUBSTR): the table code -> the code of its
// substring.  The substrings the dictionary lacks get codes in the execution's overlay
// (Dict::overlay, DictOverlays: the table's dictionary is only read), so a substring meets
// the column's own strings, string constants and GROUP BY decoding exactly as a column
// does, within the query.  An Enum's declared dictionary cannot grow.
nut_status substr_map(const Dict *cd, const std::string &cname, int off, i128 len, std::vector<int64_t> &map) {
  if (!cd) return fail(NUT_ERR_PLAN, "substring needs a string column ('" + cname + "')");
  if (cd->fixed) return fail(NUT_ERR_PLAN, "substring over the Enum column '" + cname + "' is not executed");
  if (!cd->base) return fail(NUT_ERR_INVALID_ARG, "substring over '" + cname + "': no query-local dictionary");
  Dict *d = const_cast<Dict *>(cd);  // (the execution's own overlay)
  const size_t n0 = d->size();
  map.resize(n0);
  for (size_t i = 0; i < n0; ++i) map[i] = d->intern(substr_bytes(d->at(i), off, len));
  return NUT_OK;
}
}  // namespace

nut_status build_spec(const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts, uint64_t n,
                      nut_agg_spec &s, ProgStore &store, std::vector<int> &agg_f64, GbExtra *gx) {
  memset(&s, 0, sizeof s);
  s.n = p.never ? 0 : n;
  // keys that are programs are resolved below (and packed into key words by exec_groupby)
  const bool keyprog = needs_key_progs(p);
  if (gx) {
    gx->active = keyprog;
    gx->slot.assign(p.aggs.size(), -1);
    gx->key.clear();
    gx->cu_val.assign(p.aggs.size(), nut_prog{0, nullptr});
    gx->cu_mask.assign(p.aggs.size(), nut_prog{0, nullptr});
  }
  s.nkeys = keyprog ? 0 : (int32_t)p.keys.size();
  for (size_t j = 0; j < p.keys.size() && !keyprog; ++j) {
    const nut_column *k = bound[p.keys[j]];
    if (k->type != NUT_T_I64) return fail(NUT_ERR_PLAN, "GROUP BY column '" + p.cols[p.keys[j]] + "' must be int64");
    s.keys[j] = (const int64_t *)k->data;
  }
  agg_f64.assign(p.aggs.size(), 0);
  if (p.compiled) {
    // expression mode: bind the programs' columns (first use order) and constants
    s.prog_mode = 1;
    std::vector<int> pcol(p.cols.size(), -1);
    auto bind_col = [&](int ci, int32_t &arg) -> nut_status {
      if (pcol[ci] < 0) {
        if (s.nprog_cols >= NUT_MAX_PROG_COLS) return fail(NUT_ERR_PLAN, "expressions read more than 16 columns");
        pcol[ci] = s.nprog_cols;
        s.prog_col[s.nprog_cols] = bound[ci]->data;
        s.prog_col_type[s.nprog_cols] = bound[ci]->type;
        s.nprog_cols++;
      }
      arg = pcol[ci];
      return NUT_OK;
    };
    // [I]LIKE over a dictionary column: COL, LOOKUP in a per-code byte table of the
    // dictionary strings the pattern matches (any number of them); an Enum whose codes do
    // not index a table compactly ORs equalities with the matching codes instead
    auto lower_like = [&](const PNode &n, std::vector<nut_prog_node> &v) -> nut_status {
      nut_prog_node col{NUT_P_COL, 0, 0};
      nut_status bs = bind_col(n.col, col.arg);
      if (bs) return bs;
      v.push_back(col);
      if (!dicts) {  // compile-only shape (nut_plan_prepare): an empty table
        v.push_back(nut_prog_node{NUT_P_LOOKUP, 0, 0});
        return NUT_OK;
      }
      const Dict *d = dicts[n.col];
      if (!d) return fail(NUT_ERR_PLAN, "LIKE needs a string column ('" + p.cols[n.col] + "')");
      const bool ci = n.op == P_ILIKE;
      std::vector<uint8_t> table;
      if (d->fixed) {
        int64_t lo = 0, hi = -1;
        for (const auto &kv : d->codes) {
          lo = std::min(lo, kv.second);
          hi = std::max(hi, kv.second);
        }
        if (lo < 0 || hi >= (1 << 24)) {
          size_t hits = 0;
          for (const auto &kv : d->codes) {
            if (!like_match(kv.first, n.c.s, ci)) continue;
            if (hits) v.push_back(col);
            v.push_back(nut_prog_node{NUT_P_I64, 0, kv.second});
            v.push_back(nut_prog_node{NUT_P_EQ, 0, 0});
            if (hits++) v.push_back(nut_prog_node{NUT_P_OR, 0, 0});
            if (v.size() > NUT_MAX_PROG_NODES)
              return fail(NUT_ERR_PLAN, "LIKE " + cval_str(n.c) + " over Enum column '" + p.cols[n.col] +
                                            "' (codes outside [0, 2^24)) matches too many values for one program");
          }
          if (!hits) v.push_back(nut_prog_node{NUT_P_LOOKUP, 0, 0});  // false
          return NUT_OK;
        }
        table.assign((size_t)(hi + 1), 0);
        for (const auto &kv : d->codes) table[(size_t)kv.second] = like_match(kv.first, n.c.s, ci);
      } else {
        if (d->size() > (size_t)INT32_MAX)
          return fail(NUT_ERR_PLAN, "LIKE over a dictionary of more than 2^31 strings");
        table.resize(d->size());
        for (size_t i = 0; i < d->size(); ++i) table[i] = like_match(d->at(i), n.c.s, ci);
      }
      nut_prog_node lk{NUT_P_LOOKUP, (int32_t)table.size(), 0};
      if (!table.empty()) {
        store.tables.emplace_back();
        DevBuf &t = store.tables.back();
        NUT_HIP(hipMalloc(&t.p, table.size()));
        NUT_HIP(hipMemcpy(t.p, table.data(), table.size(), hipMemcpyHostToDevice));
        lk.v = (int64_t)(uintptr_t)t.p;
      }
      v.push_back(lk);
      return NUT_OK;
    };
    // substring maps, all built before any program binds a string constant (a constant
    // compared with a substring may name a string only the substrings add)
    std::map<std::tuple<int, int, i128>, nut_prog_node> smaps;
    auto substr_node = [&](const PNode &n, nut_prog_node &out) -> nut_status {
      const auto key = std::make_tuple(n.col, n.arg, n.c.v);
      auto it = smaps.find(key);
      if (it != smaps.end()) {
        out = it->second;
        return NUT_OK;
      }
      out = nut_prog_node{NUT_P_MAP, 0, 0};  // compile-only (no dictionaries): every row -1
      if (dicts) {
        std::vector<int64_t> map;
        nut_status ms = substr_map(dicts[n.col], p.cols[n.col], n.arg, n.c.v, map);
        if (ms) return ms;
        if (map.size() > (size_t)INT32_MAX) return fail(NUT_ERR_PLAN, "substring over a dictionary of more than 2^31 strings");
        if (!map.empty()) {
          store.tables.emplace_back();
          DevBuf &t = store.tables.back();
          NUT_HIP(hipMalloc(&t.p, map.size() * 8));
          NUT_HIP(hipMemcpy(t.p, map.data(), map.size() * 8, hipMemcpyHostToDevice));
          out = nut_prog_node{NUT_P_MAP, (int32_t)map.size(), (int64_t)(uintptr_t)t.p};
        }
      }
      smaps.emplace(key, out);
      return NUT_OK;
    };
    {
      std::vector<const PProg *> all{&p.where};
      for (const PlanAgg &g : p.aggs) all.push_back(&g.val), all.push_back(&g.mask);
      for (const PProg &k : p.key_progs) all.push_back(&k);
      for (const PProg *pp : all)
        for (const PNode &nd : *pp)
          if (nd.op == P_SUBSTR) {
            nut_prog_node tmp;
            nut_status ss = substr_node(nd, tmp);
            if (ss) return ss;
          }
    }
    auto resolve = [&](const PProg &pp, nut_prog &out, const char *what, int32_t *type,
                       bool str_ok = false) -> nut_status {
      store.nodes.emplace_back();
      std::vector<nut_prog_node> &v = store.nodes.back();
      for (const PNode &n : pp) {
        nut_prog_node q{n.op, n.op == NUT_P_DATEPART ? n.arg : 0, 0};
        if (n.op == P_LIKE || n.op == P_ILIKE) {
          nut_status ls = lower_like(n, v);
          if (ls) return ls;
          continue;
        }
        if (n.op == P_SUBSTR) {  // COL, MAP (code -> the substring's code)
          nut_prog_node col{NUT_P_COL, 0, 0}, mp;
          nut_status bs = bind_col(n.col, col.arg);
          if (!bs) bs = substr_node(n, mp);
          if (bs) return bs;
          v.push_back(col);
          v.push_back(mp);
          continue;
        }
        if (n.op == NUT_P_COL) {
          if (pcol[n.col] < 0) {
            if (s.nprog_cols >= NUT_MAX_PROG_COLS) return fail(NUT_ERR_PLAN, "expressions read more than 16 columns");
            pcol[n.col] = s.nprog_cols;
            s.prog_col[s.nprog_cols] = bound[n.col]->data;
            s.prog_col_type[s.nprog_cols] = bound[n.col]->type;
            s.nprog_cols++;
          }
          q.arg = pcol[n.col];
        } else if (n.op == NUT_P_I64 && n.c.is_str) {
          // dictionary code of the compared column (-1 = absent: equal to no row);
          // dicts == NULL: compile-only (nut_plan_prepare), the code does not matter
          if (dicts) {
            if (n.col < 0 || !dicts[n.col])
              return fail(NUT_ERR_PLAN, std::string(what) + ": string constant " + cval_str(n.c) +
                                            " must be compared (= / != / IN) with a string column");
            q.v = dicts[n.col]->find(n.c.s);
          } else {
            q.v = -1;
          }
        } else if (n.op == NUT_P_I64) {
          if (n.c.v > INT64_MAX || n.c.v < INT64_MIN)
            return fail(NUT_ERR_PLAN, "integer constant " + cval_str(n.c) + " is outside int64");
          q.v = (int64_t)n.c.v;
        } else if (n.op == NUT_P_F64) {
          const double d = n.c.dec.to_f64();
          memcpy(&q.v, &d, 8);
        }
        v.push_back(q);
      }
      out.n = (int32_t)v.size();
      out.node = v.data();
      if (dicts && !str_ok) {
        nut_status cs = check_strings(p, pp, dicts, what);
        if (cs) return cs;
      }
      if (!type) return NUT_OK;
      if (nut_prog_type(&out, s.prog_col_type, NUT_MAX_PROG_COLS, type))
        return fail(NUT_ERR_PLAN, std::string(what) + ": " + nut_last_error());
      return NUT_OK;
    };
    int32_t t;
    nut_status st = NUT_OK;
    if (!p.where.empty()) {
      st = resolve(p.where, s.where, "WHERE", &t);
      if (!st && t == NUT_PT_F64) st = fail(NUT_ERR_PLAN, "WHERE: a float64 expression is not a condition");
    }
    s.naggs = 0;
    for (size_t a = 0; a < p.aggs.size() && !st; ++a) {
      const PlanAgg &g = p.aggs[a];
      if (g.distinct) {  // countUnique: its own passes (exec_groupby)
        if (!gx) continue;
        st = resolve(g.val, gx->cu_val[a], "countUnique argument", &t, true);
        if (!st && t == NUT_PT_F64) st = fail(NUT_ERR_PLAN, "countUnique of a float64 expression is not executed");
        if (!st && g.val.size() != 1 && dicts) st = check_strings(p, g.val, dicts, "countUnique argument");
        if (!st && !g.mask.empty()) st = resolve(g.mask, gx->cu_mask[a], "countUnique argument", &t);
        continue;
      }
      const int k = s.naggs++;
      if (gx) gx->slot[a] = k;
      s.agg_op[k] = g.op;
      if (g.op != NUT_AGG_COUNT) {
        // (a scan's computed projection may be a string: one column or substring of one)
        const bool str_val = p.kind != NUT_PLAN_GROUPBY && g.val.size() == 1 &&
                             (g.val[0].op == NUT_P_COL || g.val[0].op == P_SUBSTR);
        st = resolve(g.val, s.agg_val[k], "aggregate argument", &t, str_val);
        agg_f64[a] = t == NUT_PT_F64;
      }
      if (!st && !g.mask.empty()) st = resolve(g.mask, s.agg_mask[k], "aggregate argument", &t);
    }
    for (size_t j = 0; j < p.key_progs.size() && !st && keyprog && gx; ++j) {
      // a plain string column is a key of dictionary codes; computed keys are numbers
      gx->key.emplace_back();
      st = resolve(p.key_progs[j], gx->key.back(), "GROUP BY key", &t, key_dict_col(p, j) >= 0);
      if (!st && t == NUT_PT_F64)
        st = fail(NUT_ERR_PLAN, "GROUP BY key '" + p.key_text[j] + "' is float64 (keys are integers)");
    }
    if (st) return st;
  } else {
    for (const PlanPred &pr : p.preds) {
      const nut_column *col = bound[pr.col];
      const Dict *dc = dicts ? dicts[pr.col] : nullptr;
      bool any_str = pr.c.is_str;
      for (const CVal &v : pr.set) any_str = any_str || v.is_str;
      if (dc || any_str) {
        // strings: = / != / IN against dictionary codes (absent string: equal to no row)
        const std::string &cn = p.cols[pr.col];
        if (!dc) return fail(NUT_ERR_PLAN, "string constant compared with the non-string column '" + cn + "'");
        if (pr.op != NUT_EQ && pr.op != NUT_NE && pr.op < NUT_IN)
          return fail(NUT_ERR_PLAN, "ordering comparison on the string column '" + cn +
                                        "' (dictionary codes are unordered)");
        std::vector<int64_t> codes;
        for (const CVal &v : pr.op >= NUT_IN ? pr.set : std::vector<CVal>{pr.c}) {
          if (!v.is_str) return fail(NUT_ERR_PLAN, "string column '" + cn + "' compared with a number");
          const int64_t code = dc->find(v.s);
          if (code >= 0) codes.push_back(code);
        }
        const bool positive = pr.op == NUT_EQ || pr.op == NUT_IN;
        if (codes.empty()) {
          if (positive) s.n = 0;  // equal to no row; the negated form keeps every row
          continue;
        }
        s.pred_col[s.npred] = col->data;
        s.pred_type[s.npred] = NUT_T_I64;
        s.pred_op[s.npred] = positive ? NUT_IN : NUT_NOT_IN;
        s.pred_nset[s.npred] = (int32_t)codes.size();
        for (size_t j = 0; j < codes.size(); ++j) s.pred_set[s.npred][j] = codes[j];
        s.npred++;
        continue;
      }
      if (pr.op >= NUT_IN) {
        // keep the set values the column type can hold (a non-integral or out-of-range
        // constant never equals an int64)
        std::vector<int64_t> vals;
        for (const CVal &v : pr.set) {
          if (col->type == NUT_T_I64) {
            int o2;
            int64_t k;
            if (resolve_i64(NUT_EQ, v, o2, k) == V_PRED) vals.push_back(k);
          } else {
            double d = resolve_f64(v);
            int64_t bits;
            memcpy(&bits, &d, 8);
            vals.push_back(bits);
          }
        }
        if (vals.empty()) {
          if (pr.op == NUT_IN) s.n = 0;  // IN () is false; NOT IN () is true
          continue;
        }
        s.pred_col[s.npred] = col->data;
        s.pred_type[s.npred] = col->type;
        s.pred_op[s.npred] = pr.op;
        s.pred_nset[s.npred] = (int32_t)vals.size();
        for (size_t j = 0; j < vals.size(); ++j) s.pred_set[s.npred][j] = vals[j];
        s.npred++;
        continue;
      }
      if (col->type == NUT_T_I64) {
        int op;
        int64_t k;
        Verdict v = resolve_i64(pr.op, pr.c, op, k);
        if (v == V_TRUE) continue;
        if (v == V_FALSE) {
          s.n = 0;
          continue;
        }
        s.pred_col[s.npred] = col->data;
        s.pred_type[s.npred] = NUT_T_I64;
        s.pred_op[s.npred] = op;
        s.pred_i64[s.npred] = k;
      } else {
        s.pred_col[s.npred] = col->data;
        s.pred_type[s.npred] = NUT_T_F64;
        s.pred_op[s.npred] = pr.op;
        s.pred_f64[s.npred] = resolve_f64(pr.c);
      }
      s.npred++;
    }
    s.nvals = (int32_t)p.vals.size();
    for (size_t v = 0; v < p.vals.size(); ++v) {
      if (dicts && dicts[p.vals[v]])
        return fail(NUT_ERR_PLAN, "aggregate over the string column '" + p.cols[p.vals[v]] + "' (only count)");
      s.val_col[v] = bound[p.vals[v]]->data;
      s.val_type[v] = bound[p.vals[v]]->type;
    }
    s.naggs = (int32_t)p.aggs.size();
    for (size_t a = 0; a < p.aggs.size(); ++a) {
      const PlanAgg &g = p.aggs[a];
      s.agg_op[a] = g.op;
      s.agg_expr[a] = g.expr;
      for (int j = 0; j < 3; ++j) s.agg_arg[a][j] = g.arg[j];
      if (g.op != NUT_AGG_COUNT) {
        bool f = s.val_type[g.arg[0]] == NUT_T_F64;
        if (g.expr != NUT_EX_COL) {
          static const int nargs[] = {1, 2, 2, 2, 2, 3};
          for (int j = 0; j < nargs[g.expr]; ++j)
            if (s.val_type[g.arg[j]] != NUT_T_F64)
              return fail(NUT_ERR_PLAN, "fused aggregate expressions need float64 columns ('" +
                                            p.cols[p.vals[g.arg[j]]] + "' is int64)");
          f = true;
        }
        agg_f64[a] = f;
      }
    }
  }
  if (s.n == 0) {  // keep the kernels' pointer checks happy for an empty scan
    s.npred = 0;
  }
  return NUT_OK;
}


}  // namespace plan
}  // namespace nut
