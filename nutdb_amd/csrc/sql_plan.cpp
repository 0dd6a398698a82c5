// sql_plan.cpp — the SQL C ABI: parse / tokenize / unescape, plan,
// describe, prepare and execute (one table, joins, typed tables), results.  Lowering lives
// in sql_lower.cpp, execution in sql_exec_{scan,groupby,join}.cpp (sql_plan.hpp).
#include "sql_plan.hpp"

namespace {

// exact decimal of a finite double (17 significant digits: strtod gives the double back)
Decimal decimal_of(double d) {
  Decimal x;
  if (d == 0.0) return x;
  char buf[64];
  snprintf(buf, sizeof buf, "%.16e", d);  // [-]d.dddddddddddddddde[+-]XX
  const char *q = buf;
  if (*q == '-') x.neg = true, ++q;
  std::string digs;
  for (; *q && *q != 'e'; ++q)
    if (*q != '.') digs += *q;
  const int64_t ex = strtoll(q + 1, nullptr, 10);
  size_t z = 0;
  while (z < digs.size() && digs[z] == '0') ++z;
  x.digits = digs.substr(z);
  x.scale = 16 - ex;
  return x;
}

// Scalar subqueries (nut_plan.subs): run each (run(sub) executes it over the caller's
// binding), check it returned one value, and copy the plan with every placeholder constant
// replaced by that value.  A global aggregate over no rows is one row of defaults
// (ClickHouse: count / sum / min / max 0, avg NaN); a NaN (or no row) is treated as SQL
// NULL: a WHERE term comparing with it is never true; anywhere else it is rejected.
nut_status resolve_subqueries(const nut_plan &p, nut_plan &q,
                              const std::function<nut_status(const nut_plan *, nut_result **)> &run) {
  std::vector<CVal> vals(p.subs.size());
  std::vector<bool> null(p.subs.size(), false);
  for (size_t i = 0; i < p.subs.size(); ++i) {
    nut_result *r = nullptr;
    nut_status st = run(p.subs[i].get(), &r);
    if (st) return st;
    std::unique_ptr<nut_result, void (*)(nut_result *)> hold(r, nut_result_free);
    if (r->nrows > 1)
      return fail(NUT_ERR_PLAN, "scalar subquery returned " + std::to_string(r->nrows) + " rows (one expected)");
    if (r->nrows == 0 || r->host.empty() || r->host[0].empty()) {
      null[i] = true;
      continue;
    }
    const uint64_t w = r->host[0][0];
    if (r->types[0] != NUT_T_F64 && r->types[0] != NUT_T_I64)  // a dictionary code is no number
      return fail(NUT_ERR_PLAN, "scalar subquery returned a non-numeric value (type " +
                                    std::to_string(r->types[0]) + "); only int64 / float64 results compare");
    if (r->types[0] == NUT_T_F64) {
      double d;
      memcpy(&d, &w, 8);
      if (std::isnan(d)) {  // avg over no rows: comparisons with NaN are never true, as with NULL
        null[i] = true;
        continue;
      }
      if (!std::isfinite(d)) return fail(NUT_ERR_UNSUPPORTED, "scalar subquery returned an infinite value");
      vals[i].is_int = false;
      vals[i].dec = decimal_of(d);
    } else {
      vals[i].is_int = true;
      vals[i].v = (int64_t)w;
    }
  }
  q = p;
  q.subs.clear();
  bool bad_null = false;
  auto put = [&](CVal &c) {
    if (c.param < 0) return;
    if (null[c.param]) bad_null = true;
    c = vals[c.param];
  };
  for (PlanPred &pr : q.preds) {
    if ((pr.c.param >= 0 && null[pr.c.param])) {
      q.never = true;  // col <cmp> NULL: never true (the terms are ANDed)
      pr.c = CVal{};
      continue;
    }
    put(pr.c);
    for (CVal &v : pr.set) put(v);
  }
  auto prog = [&](PProg &pp) {
    for (PNode &n : pp)
      if (n.c.param >= 0) {
        put(n.c);
        n.op = n.c.is_int ? NUT_P_I64 : NUT_P_F64;
      }
  };
  prog(q.where);
  for (PProg &pp : q.proj_val) prog(pp);
  for (PProg &pp : q.proj_mask) prog(pp);
  for (PProg &pp : q.key_progs) prog(pp);
  for (PlanAgg &a : q.aggs) prog(a.val), prog(a.mask);
  for (nut_plan::JoinStep &js : q.jn) prog(js.cond);
  std::function<void(HNode &)> hv = [&](HNode &h) {
    if (h.k == H_CONST && h.param >= 0) {
      if (null[h.param]) bad_null = true;
      const CVal &v = vals[h.param];
      h.param = -1;
      if (v.is_int && v.v <= INT64_MAX && v.v >= INT64_MIN) {
        h.is_int = true;
        h.i = (int64_t)v.v;
      } else {
        h.is_int = false;
        h.f = v.is_int ? (double)v.v : v.dec.to_f64();
      }
    }
    for (HNode &k : h.kids) hv(k);
  };
  hv(q.having);
  if (bad_null) return fail(NUT_ERR_UNSUPPORTED, "a scalar subquery returned no row (NULL) where only a WHERE comparison can take it");
  return NUT_OK;
}

// The rest of a plan over its materialized derived table: the body's result (a group-by:
// host columns) bound by output name as the outer plan's table (copied into HBM by the
// call, NUT_COL_HOST).  Takes r1.
nut_status run_over_derived(nut_ctx *c, const nut_plan &p, nut_result *r1, nut_result **out) {
  struct Free {
    nut_result *r;
    ~Free() { nut_result_free(r); }
  } f{r1};
  if (r1->kind != NUT_PLAN_GROUPBY || r1->host.size() != r1->names.size())
    return fail(NUT_ERR_UNSUPPORTED, "derived table: its body did not produce a group-by result");
  std::vector<nut_column> cols;
  for (size_t j = 0; j < r1->names.size(); ++j) {
    if (r1->types[j] != NUT_T_I64 && r1->types[j] != NUT_T_F64) continue;  // (string outputs are not read back)
    cols.push_back(nut_column{r1->names[j].c_str(), r1->host[j].data(), r1->types[j] | NUT_COL_HOST});
  }
  nut_plan o = p;
  o.inner.reset();
  return nut_plan_execute(c, &o, cols.data(), (int)cols.size(), r1->nrows, 0, out);
}

// UNION ALL: the branches' results in branch order as one result — device
// columns copied after each other (scans), host columns appended (aggregates), decoded
// strings appended, NULL flags kept per column.  Column names are branch 0's; each
// column's type must agree across the branches.  Frees the parts.
nut_status concat_results(nut_ctx *c, std::vector<nut_result *> &parts, nut_result **out) {
  struct Free {
    std::vector<nut_result *> &v;
    ~Free() {
      for (nut_result *r : v) nut_result_free(r);
    }
  } f{parts};
  const nut_result &r0 = *parts[0];
  const size_t nc = r0.names.size();
  uint64_t total = 0;
  for (size_t k = 0; k < parts.size(); ++k) {
    const nut_result &r = *parts[k];
    if (r.names.size() != nc)
      return fail(NUT_ERR_PLAN, "UNION ALL: branch " + std::to_string(k + 1) + " outputs " + std::to_string(r.names.size()) +
                                    " columns, branch 1 " + std::to_string(nc));
    for (size_t j = 0; j < nc; ++j)
      if (r.types[j] != r0.types[j])
        return fail(NUT_ERR_PLAN, "UNION ALL: column " + std::to_string(j + 1) + " ('" + r0.names[j] +
                                      "') has another type in branch " + std::to_string(k + 1));
    total += r.nrows;
  }
  nut_result *u = new (std::nothrow) nut_result;
  if (!u) return fail(NUT_ERR_OOM, "UNION ALL: out of host memory");
  std::unique_ptr<nut_result, void (*)(nut_result *)> keep(u, nut_result_free);
  u->kind = r0.kind;
  u->device = c->device;
  u->nrows = total;
  u->names = r0.names;
  u->types = r0.types;
  bool any_str = false;
  for (int t : r0.types) any_str |= t == NUT_T_STR;
  if (any_str) {
    u->strs.assign(nc, {});
    for (size_t j = 0; j < nc; ++j)
      if (r0.types[j] == NUT_T_STR)
        for (const nut_result *r : parts)
          if (j < r->strs.size()) u->strs[j].insert(u->strs[j].end(), r->strs[j].begin(), r->strs[j].end());
  }
  if (r0.kind == NUT_PLAN_GROUPBY) {
    u->host.assign(nc, {});
    for (size_t j = 0; j < nc; ++j)
      for (const nut_result *r : parts)
        if (j < r->host.size()) u->host[j].insert(u->host[j].end(), r->host[j].begin(), r->host[j].end());
    *out = keep.release();
    return NUT_OK;
  }
  DeviceGuard g(c->device);
  u->dev_stride = total;
  if (total) NUT_HIP(hipMalloc(&u->dev, total * nc * 8));
  std::vector<int> vcols;  // columns with NULL flags in any branch
  for (size_t j = 0; j < nc; ++j) {
    bool v = false;
    for (const nut_result *r : parts) v |= j < r->valid_of.size() && r->valid_of[j] >= 0 && r->valid;
    u->valid_of.push_back(v ? (int)vcols.size() : -1);
    if (v) vcols.push_back((int)j);
  }
  if (!vcols.empty() && total) NUT_HIP(hipMalloc((void **)&u->valid, total * vcols.size()));
  uint64_t row = 0;
  for (const nut_result *r : parts) {
    if (r->nrows) {
      for (size_t j = 0; j < nc; ++j) {
        NUT_HIP(hipMemcpyAsync((int64_t *)u->dev + j * total + row, (const int64_t *)r->dev + j * r->dev_stride + r->dev_off,
                               r->nrows * 8, hipMemcpyDeviceToDevice, c->stream));
        if (u->valid_of[j] < 0) continue;
        uint8_t *dv = u->valid + (size_t)u->valid_of[j] * total + row;
        if (j < r->valid_of.size() && r->valid_of[j] >= 0 && r->valid)
          NUT_HIP(hipMemcpyAsync(dv, r->valid + (size_t)r->valid_of[j] * r->dev_stride + r->dev_off, r->nrows,
                                 hipMemcpyDeviceToDevice, c->stream));
        else
          NUT_HIP(hipMemsetAsync(dv, 1, r->nrows, c->stream));
      }
    }
    row += r->nrows;
  }
  NUT_HIP(hipStreamSynchronize(c->stream));  // the parts' buffers are freed on return
  *out = keep.release();
  return NUT_OK;
}

}  // namespace

extern "C" {

nut_status nut_sql_parse(const char *sql, size_t len, nut_stmt **out) {
  if (!out || (!sql && len)) return fail(NUT_ERR_INVALID_ARG, "nut_sql_parse: NULL argument");
  *out = nullptr;
  nut_stmt *s = new (std::nothrow) nut_stmt;
  if (!s) return fail(NUT_ERR_OOM, "nut_sql_parse: out of host memory");
  nut_status st = parse_into(sql ? sql : "", len, s);
  if (st) {
    delete s;
    return st;
  }
  *out = s;
  return NUT_OK;
}

int nut_stmt_kind_of(const nut_stmt *s) { return s ? (int)s->st.k : -1; }

nut_status nut_stmt_dump(const nut_stmt *s, char *buf, size_t cap, size_t *len) {
  if (!s) return fail(NUT_ERR_INVALID_ARG, "nut_stmt_dump: NULL statement");
  return put_text(dump(s->st), buf, cap, len);
}

void nut_stmt_free(nut_stmt *s) { delete s; }

nut_status nut_sql_tokenize(const char *sql, size_t len, int32_t *types, uint64_t *spans, size_t cap, size_t *ntok) {
  if (!ntok || (!sql && len) || (cap && (!types || !spans)))
    return fail(NUT_ERR_INVALID_ARG, "nut_sql_tokenize: NULL argument");
  size_t bad = 0;
  if (!valid_utf8(sql, len, &bad))
    return fail(NUT_ERR_INVALID_ARG, "sql is not valid UTF-8 (byte " + std::to_string(bad) + ")");
  Tokenizer tz(sql ? sql : "", len);
  size_t n = 0;
  for (;;) {
    Token t;
    LexError le;
    if (!tz.next_token(t, le)) {
      *ntok = n;
      return fail(NUT_ERR_PARSE, le.str());
    }
    if (n >= cap) {
      *ntok = n;
      return fail(NUT_ERR_CAPACITY, "nut_sql_tokenize: more than " + std::to_string(cap) + " tokens");
    }
    types[n] = (int32_t)t.t;
    spans[2 * n] = t.span.start;
    spans[2 * n + 1] = t.span.end;
    ++n;
    if (t.t == Tok::Eof) break;
  }
  *ntok = n;
  return NUT_OK;
}

nut_status nut_sql_unescape(const char *s, size_t len, int quote, char *out, size_t cap, size_t *out_len) {
  if (!out_len || (!s && len) || (quote != '\'' && quote != '"'))
    return fail(NUT_ERR_INVALID_ARG, "nut_sql_unescape: bad argument");
  size_t bad = 0;
  if (!valid_utf8(s, len, &bad)) return fail(NUT_ERR_INVALID_ARG, "nut_sql_unescape: input is not valid UTF-8");
  std::string r;
  ParseError pe;
  if (!unescape(sv(s ? s : "", len), (char)quote, r, pe)) return fail(NUT_ERR_PARSE, pe.msg);  // SyntaxError Display
  *out_len = r.size();
  if (r.size() > cap) return fail(NUT_ERR_CAPACITY, "nut_sql_unescape: output needs " + std::to_string(r.size()) + " bytes");
  if (!r.empty()) memcpy(out, r.data(), r.size());
  return NUT_OK;
}

nut_status nut_sql_plan(const char *sql, size_t len, nut_plan **out) {
  if (!out || (!sql && len)) return fail(NUT_ERR_INVALID_ARG, "nut_sql_plan: NULL argument");
  *out = nullptr;
  nut_stmt s;
  nut_status st = parse_into(sql ? sql : "", len, &s);
  if (st) return st;
  nut_plan *p = new (std::nothrow) nut_plan;
  if (!p) return fail(NUT_ERR_OOM, "nut_sql_plan: out of host memory");
  Lowering L;
  if (!lower(s.st, *p, L)) {
    delete p;
    return fail(NUT_ERR_PLAN, "cannot lower to an executor plan: " + L.err);
  }
  *out = p;
  return NUT_OK;
}

int nut_plan_kind_of(const nut_plan *p) { return p ? p->kind : -1; }

nut_status nut_plan_describe(const nut_plan *p, char *buf, size_t cap, size_t *len) {
  if (!p) return fail(NUT_ERR_INVALID_ARG, "nut_plan_describe: NULL plan");
  return put_text(describe(*p), buf, cap, len);
}

nut_status nut_plan_route(const nut_plan *p, const nut_column *cols, int ncols, char *buf, size_t cap, size_t *len) {
  if (!p || (ncols && !cols) || ncols < 0) return fail(NUT_ERR_INVALID_ARG, "nut_plan_route: NULL argument");
  if (p->join >= 0 || p->inner || !p->uni.empty() || !p->subs.empty())
    return fail(NUT_ERR_INVALID_ARG, "nut_plan_route: single-table plans without subqueries or UNION only");
  nut_plan sq;
  if (p->star) {
    std::vector<std::string> names;
    for (int i = 0; i < ncols; ++i)
      if (cols[i].name) names.push_back(cols[i].name);
    p = expand_star(*p, names, sq);
  }
  std::vector<const nut_column *> bound(p->cols.size());
  for (size_t i = 0; i < p->cols.size(); ++i) {
    bound[i] = bind(*p, (int)i, cols, ncols);
    if (!bound[i]) return fail(NUT_ERR_INVALID_ARG, "nut_plan_route: column '" + p->cols[i] + "' is not bound");
    if (bound[i]->type != NUT_T_I64 && bound[i]->type != NUT_T_F64)
      return fail(NUT_ERR_INVALID_ARG, "nut_plan_route: column '" + p->cols[i] + "' has an unknown type");
  }
  std::string route;
  if (p->kind == NUT_PLAN_GROUPBY) {
    nut_agg_spec s;
    ProgStore store;
    std::vector<int> agg_f64;
    GbExtra gx;
    // float64 key columns are grouped on int64 key words (exec_groupby)
    std::deque<nut_column> words;
    int nf = 0;
    for (int k : p->keys)
      if (k >= 0 && bound[k]->type == NUT_T_F64) {
        words.push_back(nut_column{bound[k]->name, nullptr, NUT_T_I64});
        bound[k] = &words.back();
        ++nf;
      }
    nut_status st = build_spec(*p, bound.data(), nullptr, 0, s, store, agg_f64, &gx);
    if (st) return st;
    route = gx.active ? "packed-groupby" : p->compiled ? "expr-groupby" : "fused-groupby";
    if (nf) route += " (float64 key words)";
  } else {
    ScanRoute r;
    nut_status st = scan_route(*p, bound.data(), nullptr, &r);
    if (st) return st;
    route = scan_route_name(r);
    if (r == S_RERUN_EXPR) {  // and where the rerun lands
      nut_plan q = *p;
      std::vector<PProg> cs;
      for (const PlanPred &pr : p->preds) cs.push_back(pred_prog(pr));
      q.compiled = true;
      q.preds.clear();
      q.where = and_all(cs);
      st = scan_route(q, bound.data(), nullptr, &r);
      if (st) return st;
      route += std::string(" -> ") + scan_route_name(r);
    }
  }
  return put_text(route, buf, cap, len);
}

void nut_plan_free(nut_plan *p) { delete p; }

nut_status nut_plan_execute(nut_ctx *c, const nut_plan *p, const nut_column *cols, int ncols, uint64_t nrows,
                            uint64_t group_hint, nut_result **out) {
  if (p && out && !p->uni.empty()) {  // UNION ALL: every branch over the same columns
    *out = nullptr;
    std::vector<nut_result *> parts;
    for (const auto &b : p->uni) {
      nut_result *r = nullptr;
      nut_status st = nut_plan_execute(c, b.get(), cols, ncols, nrows, group_hint, &r);
      if (st) {
        for (nut_result *x : parts) nut_result_free(x);
        return st;
      }
      parts.push_back(r);
    }
    return concat_results(c, parts, out);
  }
  if (!c || !p || !out || (ncols && !cols) || ncols < 0) return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute: NULL argument");
  *out = nullptr;
  if (p->inner) {  // a materialized derived table: its body first, over the caller's columns
    if (p->inner->join >= 0) return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute: the derived table has a JOIN (nut_plan_execute2)");
    nut_result *r1 = nullptr;
    nut_status st = nut_plan_execute(c, p->inner.get(), cols, ncols, nrows, group_hint, &r1);
    return st ? st : run_over_derived(c, *p, r1, out);
  }
  if (p->join >= 0) return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute: the plan has a JOIN (nut_plan_execute2)");
  if (!p->subs.empty()) {  // scalar subqueries first, over the same columns
    nut_plan q;
    nut_status st = resolve_subqueries(*p, q, [&](const nut_plan *sp, nut_result **r) {
      return nut_plan_execute(c, sp, cols, ncols, nrows, 1, r);
    });
    return st ? st : nut_plan_execute(c, &q, cols, ncols, nrows, group_hint, out);
  }
  nut_plan sq;
  if (p->star) {
    std::vector<std::string> names;
    for (int i = 0; i < ncols; ++i)
      if (cols[i].name) names.push_back(cols[i].name);
    if (names.empty()) return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute: SELECT * over no columns");
    p = expand_star(*p, names, sq);
  }
  DeviceGuard g0(c->device);
  HostStage hs;
  nut_status hst = stage_host(c, cols, ncols, nrows, hs, &cols);
  if (hst) return hst;
  std::vector<const nut_column *> bound(p->cols.size());
  for (size_t i = 0; i < p->cols.size(); ++i) {
    bound[i] = bind(*p, (int)i, cols, ncols);
    if (!bound[i]) return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute: column '" + p->cols[i] + "' is not bound");
    if (bound[i]->type != NUT_T_I64 && bound[i]->type != NUT_T_F64)
      return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute: column '" + p->cols[i] + "' has an unknown type");
    if (nrows && !bound[i]->data) return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute: column '" + p->cols[i] + "' is NULL");
  }
  nut_result *r = new (std::nothrow) nut_result;
  if (!r) return fail(NUT_ERR_OOM, "nut_plan_execute: out of host memory");
  r->kind = p->kind;
  r->device = c->device;
  DeviceGuard g(c->device);
  const std::vector<const Dict *> nodict(p->cols.size(), nullptr);  // raw columns carry no strings
  nut_status st = p->kind == NUT_PLAN_GROUPBY ? exec_groupby(c, *p, bound.data(), nodict.data(), nrows, group_hint, r)
                                              : exec_scan(c, *p, bound.data(), nodict.data(), nrows, r);
  if (st) {
    nut_result_free(r);
    return st;
  }
  *out = r;
  return NUT_OK;
}

nut_status nut_plan_execute2(nut_ctx *c, const nut_plan *p, const nut_column *left, int nleft, uint64_t lrows,
                             const nut_column *right, int nright, uint64_t rrows, uint64_t group_hint,
                             nut_result **out) {
  if (!c || !p || !out || (nleft && !left) || (nright && !right) || nleft < 0 || nright < 0)
    return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute2: NULL argument");
  if (!p->uni.empty()) {  // UNION ALL of two branches: branch k over table k
    const nut_column *tabs[2] = {left, right};
    const int nc[2] = {nleft, nright};
    const uint64_t nr[2] = {lrows, rrows};
    return nut_plan_executen(c, p, tabs, nc, nr, 2, group_hint, out);
  }
  if (p->inner) {  // a materialized derived table over the two tables, then the rest over it
    *out = nullptr;
    nut_result *r1 = nullptr;
    nut_status st = nut_plan_execute2(c, p->inner.get(), left, nleft, lrows, right, nright, rrows, group_hint, &r1);
    return st ? st : run_over_derived(c, *p, r1, out);
  }
  if (p->join < 0) return nut_plan_execute(c, p, left, nleft, lrows, group_hint, out);
  if (!p->subs.empty()) {  // scalar subqueries first, over the FROM table (left)
    nut_plan q;
    nut_status st = resolve_subqueries(*p, q, [&](const nut_plan *sp, nut_result **r) {
      return nut_plan_execute(c, sp, left, nleft, lrows, 1, r);
    });
    return st ? st : nut_plan_execute2(c, &q, left, nleft, lrows, right, nright, rrows, group_hint, out);
  }
  if (p->jn.size() == 1) {  // one JOIN run as a chain step (ON filters, EXISTS / IN)
    const nut_column *tabs[2] = {left, right};
    const int nc[2] = {nleft, nright};
    const uint64_t nr[2] = {lrows, rrows};
    return nut_plan_executen(c, p, tabs, nc, nr, 2, group_hint, out);
  }
  if (!p->jn.empty()) return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute2: the plan joins several tables (nut_plan_executen)");
  *out = nullptr;
  DeviceGuard g(c->device);
  HostStage hl, hr;
  nut_status st = stage_host(c, left, nleft, lrows, hl, &left);
  if (!st) st = stage_host(c, right, nright, rrows, hr, &right);
  if (st) return st;
  nut_result *r = new (std::nothrow) nut_result;
  if (!r) return fail(NUT_ERR_OOM, "nut_plan_execute2: out of host memory");
  r->kind = p->kind;
  r->device = c->device;
  st = exec_join(c, *p, left, nleft, lrows, right, nright, rrows, group_hint, r);
  if (st) {
    nut_result_free(r);
    return st;
  }
  *out = r;
  return NUT_OK;
}

nut_status nut_plan_executen(nut_ctx *c, const nut_plan *p, const nut_column *const *tables, const int *ncols,
                             const uint64_t *nrows, int ntables, uint64_t group_hint, nut_result **out) {
  if (!c || !p || !out || !tables || !ncols || !nrows || ntables < 1)
    return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: NULL argument");
  if (!p->uni.empty()) {  // UNION ALL: branch k over table k (or every branch over table 0)
    if (ntables != 1 && (size_t)ntables != p->uni.size())
      return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: a UNION ALL of " + std::to_string(p->uni.size()) +
                                           " branches takes one table per branch (or one for all)");
    *out = nullptr;
    std::vector<nut_result *> parts;
    for (size_t k = 0; k < p->uni.size(); ++k) {
      const int t = ntables == 1 ? 0 : (int)k;
      nut_result *r = nullptr;
      nut_status st = nut_plan_execute(c, p->uni[k].get(), tables[t], ncols[t], nrows[t], group_hint, &r);
      if (st) {
        for (nut_result *x : parts) nut_result_free(x);
        return st;
      }
      parts.push_back(r);
    }
    return concat_results(c, parts, out);
  }
  if (p->inner) {  // a materialized derived table over the tables, then the rest over it
    *out = nullptr;
    nut_result *r1 = nullptr;
    nut_status st = nut_plan_executen(c, p->inner.get(), tables, ncols, nrows, ntables, group_hint, &r1);
    return st ? st : run_over_derived(c, *p, r1, out);
  }
  if (p->jn.empty()) {
    if (ntables == 1) return nut_plan_execute(c, p, tables[0], ncols[0], nrows[0], group_hint, out);
    if (ntables == 2)
      return nut_plan_execute2(c, p, tables[0], ncols[0], nrows[0], tables[1], ncols[1], nrows[1], group_hint, out);
    return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: the plan joins fewer tables");
  }
  if (!p->subs.empty()) {  // scalar subqueries first, over the FROM table (table 0)
    nut_plan q;
    nut_status st = resolve_subqueries(*p, q, [&](const nut_plan *sp, nut_result **r) {
      return nut_plan_execute(c, sp, tables[0], ncols[0], nrows[0], 1, r);
    });
    return st ? st : nut_plan_executen(c, &q, tables, ncols, nrows, ntables, group_hint, out);
  }
  *out = nullptr;
  DeviceGuard g(c->device);
  std::deque<HostStage> hs(ntables);
  std::vector<const nut_column *> tabs(tables, tables + ntables);
  for (int k = 0; k < ntables; ++k) {
    if (ncols[k] && !tables[k]) return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: NULL table");
    nut_status hst = stage_host(c, tables[k], ncols[k], nrows[k], hs[k], &tabs[k]);
    if (hst) return hst;
  }
  nut_result *r = new (std::nothrow) nut_result;
  if (!r) return fail(NUT_ERR_OOM, "nut_plan_executen: out of host memory");
  r->kind = p->kind;
  r->device = c->device;
  nut_status st = exec_joinn(c, *p, tabs.data(), ncols, nrows, ntables, group_hint, r);
  if (st) {
    nut_result_free(r);
    return st;
  }
  *out = r;
  return NUT_OK;
}

nut_status nut_plan_prepare(const nut_plan *p, const nut_column *cols, int ncols) {
  if (!p || (ncols && !cols) || ncols < 0) return fail(NUT_ERR_INVALID_ARG, "nut_plan_prepare: NULL argument");
  if (p->inner) return nut_plan_prepare(p->inner.get(), cols, ncols);  // (the rest compiles when it runs)
  for (const auto &b : p->uni) {  // UNION ALL: every branch whose columns are all given
    bool all = true;
    for (const std::string &n : b->cols) {
      bool found = false;
      for (int i = 0; i < ncols && !found; ++i) found = cols[i].name && n == cols[i].name;
      all = all && found;
    }
    if (all) {
      nut_status st = nut_plan_prepare(b.get(), cols, ncols);
      if (st) return st;
    }
  }
  if (!p->uni.empty()) return NUT_OK;
  if (!p->compiled) return NUT_OK;  // precompiled kernels only
  // scalar subqueries: their values (int64 or f64 constants) decide the program types, so
  // the shape is compiled when the plan executes with the values in place
  if (!p->subs.empty()) return NUT_OK;
  nut_plan sq;
  if (p->star) {
    std::vector<std::string> names;
    for (int i = 0; i < ncols; ++i)
      if (cols[i].name) names.push_back(cols[i].name);
    p = expand_star(*p, names, sq);
  }
  std::vector<const nut_column *> bound(p->cols.size());
  std::vector<nut_column> typed(p->cols.size());
  for (size_t i = 0; i < p->cols.size(); ++i) {
    bound[i] = bind(*p, (int)i, cols, ncols);
    if (!bound[i]) return fail(NUT_ERR_INVALID_ARG, "nut_plan_prepare: column '" + p->cols[i] + "' is not bound");
    typed[i] = *bound[i];
    typed[i].type &= ~NUT_COL_HOST;  // only the type matters here
    bound[i] = &typed[i];
    if (bound[i]->type != NUT_T_I64 && bound[i]->type != NUT_T_F64)
      return fail(NUT_ERR_INVALID_ARG, "nut_plan_prepare: column '" + p->cols[i] + "' has an unknown type");
  }
  nut_agg_spec s;
  ProgStore store;
  std::vector<int> agg_f64;
  nut_status st = build_spec(*p, bound.data(), nullptr, 0, s, store, agg_f64);
  if (st) return st;
  st = p->kind == NUT_PLAN_GROUPBY ? nut_groupby_jit_compile(&s) : nut_select_jit_compile(&s);
  // computed projections: their evaluation kernels (groups of NUT_MAX_AGGS, as executed)
  std::vector<size_t> comp;
  for (size_t j = 0; j < p->projs.size(); ++j)
    if (computed_proj(*p, j)) comp.push_back(j);
  for (size_t g0 = 0; g0 < comp.size() && !st; g0 += NUT_MAX_AGGS) {
    nut_plan q;
    q.compiled = true;
    q.cols = p->cols;
    for (size_t t = g0; t < comp.size() && t < g0 + NUT_MAX_AGGS; ++t) {
      PlanAgg a{};
      a.op = NUT_AGG_SUM;
      a.val = p->proj_val[comp[t]];
      a.mask = p->proj_mask[comp[t]];
      q.aggs.push_back(std::move(a));
    }
    nut_agg_spec es;
    ProgStore estore;
    std::vector<int> f64;
    st = build_spec(q, bound.data(), nullptr, 0, es, estore, f64);
    if (!st) st = nut_eval_jit_compile(&es);
  }
  return st;
}

nut_status nut_table_execute(nut_ctx *c, nut_table *t, const nut_plan *p, uint64_t group_hint, nut_result **out) {
  if (!c || !t || !p || !out) return fail(NUT_ERR_INVALID_ARG, "nut_table_execute: NULL argument");
  *out = nullptr;
  if (!p->uni.empty()) {  // UNION ALL: every branch over the one table
    std::vector<nut_table *> ts(p->uni.size(), t);
    return nut_table_executen(c, ts.data(), (int)ts.size(), p, group_hint, out);
  }
  if (p->inner) {  // a materialized derived table (string outputs of its body stay unread)
    if (p->inner->join >= 0) return fail(NUT_ERR_INVALID_ARG, "nut_table_execute: the derived table has a JOIN (nut_table_execute2)");
    nut_result *r1 = nullptr;
    nut_status st = nut_table_execute(c, t, p->inner.get(), group_hint, &r1);
    return st ? st : run_over_derived(c, *p, r1, out);
  }
  if (t->ragged()) return fail(NUT_ERR_INVALID_ARG, "nut_table_execute: table '" + t->name + "' has ragged columns");
  if (t->device >= 0 && t->device != c->device)
    return fail(NUT_ERR_INVALID_ARG, "nut_table_execute: the table lives on another device");
  const uint64_t nrows = t->rows();
  if (!p->subs.empty()) {  // scalar subqueries first, over the same table
    nut_plan q;
    nut_status st = resolve_subqueries(*p, q, [&](const nut_plan *sp, nut_result **r) {
      return nut_table_execute(c, t, sp, 1, r);
    });
    return st ? st : nut_table_execute(c, t, &q, group_hint, out);
  }
  nut_plan sq;
  if (p->star) {
    std::vector<std::string> names;
    for (const TCol &x : t->cols) names.push_back(x.name);
    if (names.empty()) return fail(NUT_ERR_INVALID_ARG, "nut_table_execute: SELECT * over no columns");
    p = expand_star(*p, names, sq);
  }
  std::vector<nut_column> cols(p->cols.size());
  std::vector<const nut_column *> bound(p->cols.size());
  std::vector<const Dict *> dicts(p->cols.size(), nullptr);
  DictOverlays ov;  // the query's own view of the table's dictionary (substring results)
  for (size_t i = 0; i < p->cols.size(); ++i) {
    const TCol *tc = nullptr;
    for (const TCol &x : t->cols)
      if (ieq(x.name, p->cols[i])) tc = &x;
    const size_t dot = p->cols[i].find('.');  // a qualified name: its bare column otherwise
    for (const TCol &x : t->cols)
      if (!tc && dot != std::string::npos && ieq(x.name, sv(p->cols[i]).substr(dot + 1))) tc = &x;
    if (!tc) return fail(NUT_ERR_PLAN, "table '" + t->name + "' has no column '" + p->cols[i] + "'");
    cols[i] = nut_column{tc->name.c_str(), tc->dev, tc->exec_type};
    bound[i] = &cols[i];
    dicts[i] = ov.of(tc->dict);
  }
  nut_result *r = new (std::nothrow) nut_result;
  if (!r) return fail(NUT_ERR_OOM, "nut_table_execute: out of host memory");
  r->kind = p->kind;
  r->device = c->device;
  DeviceGuard g(c->device);
  nut_status st = p->kind == NUT_PLAN_GROUPBY ? exec_groupby(c, *p, bound.data(), dicts.data(), nrows, group_hint, r)
                                              : exec_scan(c, *p, bound.data(), dicts.data(), nrows, r);
  if (st) {
    nut_result_free(r);
    return st;
  }
  *out = r;
  return NUT_OK;
}

nut_status nut_table_execute2(nut_ctx *c, nut_table *left, nut_table *right, const nut_plan *p, uint64_t group_hint,
                              nut_result **out) {
  if (!c || !left || !right || !p || !out) return fail(NUT_ERR_INVALID_ARG, "nut_table_execute2: NULL argument");
  if (!p->uni.empty()) {  // UNION ALL of two branches: branch k over table k
    nut_table *ts[2] = {left, right};
    return nut_table_executen(c, ts, 2, p, group_hint, out);
  }
  if (p->inner) {
    *out = nullptr;
    nut_result *r1 = nullptr;
    nut_status st = nut_table_execute2(c, left, right, p->inner.get(), group_hint, &r1);
    return st ? st : run_over_derived(c, *p, r1, out);
  }
  if (p->join < 0) return nut_table_execute(c, left, p, group_hint, out);
  if (!p->jn.empty()) {  // one JOIN run as a chain step (ON filters, EXISTS / IN)
    nut_table *const tabs[2] = {left, right};
    return nut_table_executen(c, tabs, 2, p, group_hint, out);
  }
  if (!p->subs.empty()) {  // scalar subqueries first, over the FROM table (left)
    nut_plan q;
    nut_status st = resolve_subqueries(*p, q, [&](const nut_plan *sp, nut_result **r) {
      return nut_table_execute(c, left, sp, 1, r);
    });
    return st ? st : nut_table_execute2(c, left, right, &q, group_hint, out);
  }
  *out = nullptr;
  std::vector<nut_column> cols[2];
  std::vector<const Dict *> dicts[2];
  DictOverlays ov;
  nut_table *t2[2] = {left, right};
  for (int k = 0; k < 2; ++k) {
    nut_table *t = t2[k];
    if (t->ragged()) return fail(NUT_ERR_INVALID_ARG, "nut_table_execute2: table '" + t->name + "' has ragged columns");
    if (t->device >= 0 && t->device != c->device)
      return fail(NUT_ERR_INVALID_ARG, "nut_table_execute2: table '" + t->name + "' lives on another device");
    for (const TCol &x : t->cols) {
      cols[k].push_back(nut_column{x.name.c_str(), x.dev, x.exec_type});
      dicts[k].push_back(ov.of(x.dict));
    }
  }
  nut_result *r = new (std::nothrow) nut_result;
  if (!r) return fail(NUT_ERR_OOM, "nut_table_execute2: out of host memory");
  r->kind = p->kind;
  r->device = c->device;
  DeviceGuard g(c->device);
  nut_status st = exec_join(c, *p, cols[0].data(), (int)cols[0].size(), left->rows(), cols[1].data(),
                            (int)cols[1].size(), right->rows(), group_hint, r, dicts[0].data(), dicts[1].data());
  if (st) {
    nut_result_free(r);
    return st;
  }
  *out = r;
  return NUT_OK;
}

nut_status nut_table_executen(nut_ctx *c, nut_table *const *tables, int ntables, const nut_plan *p,
                              uint64_t group_hint, nut_result **out) {
  if (!c || !tables || ntables < 1 || !p || !out) return fail(NUT_ERR_INVALID_ARG, "nut_table_executen: NULL argument");
  for (int k = 0; k < ntables; ++k)
    if (!tables[k]) return fail(NUT_ERR_INVALID_ARG, "nut_table_executen: NULL table");
  if (!p->uni.empty()) {  // UNION ALL: branch k over table k (or every branch over table 0)
    if (ntables != 1 && (size_t)ntables != p->uni.size())
      return fail(NUT_ERR_INVALID_ARG, "nut_table_executen: a UNION ALL of " + std::to_string(p->uni.size()) +
                                           " branches takes one table per branch (or one for all)");
    *out = nullptr;
    std::vector<nut_result *> parts;
    for (size_t k = 0; k < p->uni.size(); ++k) {
      nut_result *r = nullptr;
      nut_status st = nut_table_execute(c, tables[ntables == 1 ? 0 : k], p->uni[k].get(), group_hint, &r);
      if (st) {
        for (nut_result *x : parts) nut_result_free(x);
        return st;
      }
      parts.push_back(r);
    }
    return concat_results(c, parts, out);
  }
  if (p->inner) {
    *out = nullptr;
    nut_result *r1 = nullptr;
    nut_status st = nut_table_executen(c, tables, ntables, p->inner.get(), group_hint, &r1);
    return st ? st : run_over_derived(c, *p, r1, out);
  }
  if (p->jn.empty()) {
    if (ntables == 1) return nut_table_execute(c, tables[0], p, group_hint, out);
    if (ntables == 2) return nut_table_execute2(c, tables[0], tables[1], p, group_hint, out);
    return fail(NUT_ERR_INVALID_ARG, "nut_table_executen: the plan joins fewer tables");
  }
  if (!p->subs.empty()) {  // scalar subqueries first, over the FROM table (table 0)
    nut_plan q;
    nut_status st = resolve_subqueries(*p, q, [&](const nut_plan *sp, nut_result **r) {
      return nut_table_execute(c, tables[0], sp, 1, r);
    });
    return st ? st : nut_table_executen(c, tables, ntables, &q, group_hint, out);
  }
  *out = nullptr;
  std::vector<std::vector<nut_column>> cols(ntables);
  std::vector<std::vector<const Dict *>> dicts(ntables);
  DictOverlays ov;
  std::vector<const nut_column *> tabs(ntables);
  std::vector<const Dict *const *> tdicts(ntables);
  std::vector<int> ncols(ntables);
  std::vector<uint64_t> nrows(ntables);
  for (int k = 0; k < ntables; ++k) {
    nut_table *t = tables[k];
    if (t->ragged()) return fail(NUT_ERR_INVALID_ARG, "nut_table_executen: table '" + t->name + "' has ragged columns");
    if (t->device >= 0 && t->device != c->device)
      return fail(NUT_ERR_INVALID_ARG, "nut_table_executen: table '" + t->name + "' lives on another device");
    for (const TCol &x : t->cols) {
      cols[k].push_back(nut_column{x.name.c_str(), x.dev, x.exec_type});
      dicts[k].push_back(ov.of(x.dict));
    }
    tabs[k] = cols[k].data();
    tdicts[k] = dicts[k].data();
    ncols[k] = (int)cols[k].size();
    nrows[k] = t->rows();
  }
  nut_result *r = new (std::nothrow) nut_result;
  if (!r) return fail(NUT_ERR_OOM, "nut_table_executen: out of host memory");
  r->kind = p->kind;
  r->device = c->device;
  DeviceGuard g(c->device);
  nut_status st = exec_joinn(c, *p, tabs.data(), ncols.data(), nrows.data(), ntables, group_hint, r, tdicts.data());
  if (st) {
    nut_result_free(r);
    return st;
  }
  *out = r;
  return NUT_OK;
}

nut_status nut_result_string(const nut_result *r, int j, uint64_t row, const char **str, size_t *len) {
  if (!r || j < 0 || j >= (int)r->names.size() || !str || !len)
    return fail(NUT_ERR_INVALID_ARG, "nut_result_string: bad argument");
  if (r->types[j] != NUT_T_STR || (size_t)j >= r->strs.size())
    return fail(NUT_ERR_INVALID_ARG, "nut_result_string: column is not a string column");
  if (row >= r->nrows) return fail(NUT_ERR_INVALID_ARG, "nut_result_string: row out of range");
  const std::string &v = r->strs[j][row];
  *str = v.data();
  *len = v.size();
  return NUT_OK;
}

nut_status nut_result_shape(const nut_result *r, uint64_t *nrows, int *ncols) {
  if (!r) return fail(NUT_ERR_INVALID_ARG, "nut_result_shape: NULL result");
  if (nrows) *nrows = r->nrows;
  if (ncols) *ncols = (int)r->names.size();
  return NUT_OK;
}

nut_status nut_result_column(const nut_result *r, int j, int *type, const char **name) {
  if (!r || j < 0 || j >= (int)r->names.size()) return fail(NUT_ERR_INVALID_ARG, "nut_result_column: bad column");
  if (type) *type = r->types[j];
  if (name) *name = r->names[j].c_str();
  return NUT_OK;
}

nut_status nut_result_to_host(const nut_result *r, int j, void *dst, uint64_t cap) {
  if (!r || j < 0 || j >= (int)r->names.size()) return fail(NUT_ERR_INVALID_ARG, "nut_result_to_host: bad column");
  if (r->nrows > cap) return fail(NUT_ERR_CAPACITY, "nut_result_to_host: capacity < " + std::to_string(r->nrows));
  if (r->nrows == 0) return NUT_OK;
  if (!dst) return fail(NUT_ERR_INVALID_ARG, "nut_result_to_host: NULL dst");
  if (r->kind == NUT_PLAN_GROUPBY) {
    if (r->types[j] == NUT_T_STR)
      return fail(NUT_ERR_INVALID_ARG, "nut_result_to_host: string column (use nut_result_string)");
    memcpy(dst, r->host[j].data(), r->nrows * 8);
    return NUT_OK;
  }
  if (r->types[j] == NUT_T_STR) return fail(NUT_ERR_INVALID_ARG, "nut_result_to_host: string column (use nut_result_string)");
  DeviceGuard g(r->device);
  NUT_HIP(hipMemcpy(dst, (const int64_t *)r->dev + (uint64_t)j * r->dev_stride + r->dev_off, r->nrows * 8,
                    hipMemcpyDeviceToHost));
  return NUT_OK;
}

nut_status nut_result_device_column(const nut_result *r, int j, const void **dev) {
  if (!r || !dev || j < 0 || j >= (int)r->names.size())
    return fail(NUT_ERR_INVALID_ARG, "nut_result_device_column: bad argument");
  if (r->kind == NUT_PLAN_GROUPBY)
    return fail(NUT_ERR_UNSUPPORTED, "nut_result_device_column: group results live on the host");
  *dev = r->dev ? (const void *)((const int64_t *)r->dev + (uint64_t)j * r->dev_stride + r->dev_off) : nullptr;
  return NUT_OK;
}

nut_status nut_result_device(const nut_result *r, const void **dev) {
  if (!r || !dev) return fail(NUT_ERR_INVALID_ARG, "nut_result_device: NULL argument");
  if (r->kind == NUT_PLAN_GROUPBY) return fail(NUT_ERR_UNSUPPORTED, "nut_result_device: group results live on the host");
  *dev = r->dev ? (const void *)((const int64_t *)r->dev + r->dev_off) : nullptr;
  return NUT_OK;
}

void nut_result_free(nut_result *r) {
  if (!r) return;
  if (r->dev) {
    DeviceGuard g(r->device);
    (void)hipFree(r->dev);
  }
  if (r->valid) {
    DeviceGuard g(r->device);
    (void)hipFree(r->valid);
  }
  delete r;
}

nut_status nut_result_validity(const nut_result *r, int j, const uint8_t **dev) {
  if (!r || !dev || j < 0 || j >= (int)r->names.size()) return fail(NUT_ERR_INVALID_ARG, "nut_result_validity: bad argument");
  const int v = j < (int)r->valid_of.size() ? r->valid_of[j] : -1;
  *dev = v >= 0 && r->valid ? r->valid + (uint64_t)v * r->dev_stride + r->dev_off : nullptr;
  return NUT_OK;
}

nut_status nut_result_validity_to_host(const nut_result *r, int j, uint8_t *dst, uint64_t cap) {
  const uint8_t *dev = nullptr;
  nut_status s = nut_result_validity(r, j, &dev);
  if (s) return s;
  if (r->nrows > cap) return fail(NUT_ERR_CAPACITY, "nut_result_validity_to_host: capacity < " + std::to_string(r->nrows));
  if (r->nrows == 0) return NUT_OK;
  if (!dst) return fail(NUT_ERR_INVALID_ARG, "nut_result_validity_to_host: NULL dst");
  if (!dev) {
    memset(dst, 1, r->nrows);
    return NUT_OK;
  }
  DeviceGuard g(r->device);
  NUT_HIP(hipMemcpy(dst, dev, r->nrows, hipMemcpyDeviceToHost));
  return NUT_OK;
}

}  // extern "C"

