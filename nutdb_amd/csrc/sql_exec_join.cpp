// sql_exec_join.cpp — executing JOIN plans: one clause of any type (nut_plan_execute2) and
// chains (nut_plan_executen), predicate pushdown, gathers into the joined table.
#include <array>

#include "sql_plan.hpp"

namespace nut {
namespace plan {


// A plan with a JOIN (nut_plan_execute2): hash join on the ON columns, gathers of every
// plan column through the join index, then the plan's scan / group-by on the joined rows.
// conjuncts of a boolean program: `A AND B` splits into A's and B's conjuncts
void split_and(const PProg &pp, std::vector<PProg> &out) {
  if (pp.empty()) return;
  if (pp.back().op != NUT_P_AND) {
    out.push_back(pp);
    return;
  }
  // subtree starts: the AND's two operands are the last two subtrees before it
  std::vector<size_t> st;
  for (size_t i = 0; i + 1 < pp.size(); ++i) {
    const int op = pp[i].op;
    const int k = pnode_arity(op);
    size_t start = i;
    for (int j = 0; j < k; ++j) {
      start = st.back();
      st.pop_back();
    }
    st.push_back(start);
  }
  if (st.size() != 2) {  // malformed: keep whole
    out.push_back(pp);
    return;
  }
  split_and(PProg(pp.begin(), pp.begin() + st[1]), out);
  split_and(PProg(pp.begin() + st[1], pp.end() - 1), out);
}

PProg and_all(const std::vector<PProg> &cs) {
  PProg r;
  for (size_t i = 0; i < cs.size(); ++i) {
    r.insert(r.end(), cs[i].begin(), cs[i].end());
    if (i) {
      PNode a;
      a.op = NUT_P_AND;
      r.push_back(a);
    }
  }
  return r;
}

// a fused-mode predicate as a program: col <cmp> c, or an OR / AND of equalities (IN)
PProg pred_prog(const PlanPred &pr) {
  auto konst = [&](const CVal &c) {
    PNode n;
    n.op = c.is_int || c.is_str ? NUT_P_I64 : NUT_P_F64;
    n.c = c;
    n.col = pr.col;  // string constants take the compared column's dictionary
    return n;
  };
  PNode col;
  col.op = NUT_P_COL;
  col.col = pr.col;
  PProg r;
  if (pr.op < NUT_IN) {
    r = {col, konst(pr.c)};
    PNode cmp;
    cmp.op = NUT_P_LT + pr.op;
    r.push_back(cmp);
    return r;
  }
  for (size_t i = 0; i < pr.set.size(); ++i) {
    r.push_back(col);
    r.push_back(konst(pr.set[i]));
    PNode cmp;
    cmp.op = pr.op == NUT_IN ? NUT_P_EQ : NUT_P_NE;
    r.push_back(cmp);
    if (i) {
      PNode j;
      j.op = pr.op == NUT_IN ? NUT_P_OR : NUT_P_AND;
      r.push_back(j);
    }
  }
  return r;
}

// an aggregate's row mask gains (column m != 0) [AND its own mask]: outer joins' NULL rows
void add_null_mask(PlanAgg &a, int m) {
  const bool had = !a.mask.empty();
  PNode col;
  col.op = NUT_P_COL;
  col.col = m;
  a.mask.push_back(col);
  emit_int(a.mask, 0);
  emit(a.mask, NUT_P_NE);
  if (had) emit(a.mask, NUT_P_AND);
}

// A scan's projections that read NULL-extended tables (outer joins): each becomes a
// computed projection masked by those tables' matched flags — SQL NULL on the rows where a
// table has no row (an expression over a NULL is NULL).  nullable(ci): the column's table
// is NULL-extended; mflag(ci): the plan column of that table's matched flag.  A fused scan
// turns into an expression-mode one (its comparisons into the WHERE program).
bool mask_null_projections(nut_plan &q, const std::function<bool(int)> &nullable, const std::function<int(int)> &mflag) {
  bool any = false;
  for (size_t j = 0; j < q.projs.size(); ++j) {
    std::vector<int> read;
    if (q.projs[j] >= 0) read.push_back(q.projs[j]);
    for (const PProg *pp : {&q.proj_val[j], &q.proj_mask[j]})
      for (const PNode &nd : *pp)
        if (reads_col(nd.op)) read.push_back(nd.col);
    std::vector<int> flags;
    for (int ci : read)
      if (nullable(ci)) {
        const int f = mflag(ci);
        if (std::find(flags.begin(), flags.end(), f) == flags.end()) flags.push_back(f);
      }
    if (flags.empty()) continue;
    any = true;
    if (q.projs[j] >= 0) {
      PNode col;
      col.op = NUT_P_COL;
      col.col = q.projs[j];
      q.proj_val[j] = PProg{col};
      q.projs[j] = -1;
    }
    for (int f : flags) {
      const bool had = !q.proj_mask[j].empty();
      PNode col;
      col.op = NUT_P_COL;
      col.col = f;
      q.proj_mask[j].push_back(col);
      emit_int(q.proj_mask[j], 0);
      emit(q.proj_mask[j], NUT_P_NE);
      if (had) emit(q.proj_mask[j], NUT_P_AND);
    }
  }
  if (any && !q.compiled) {
    std::vector<PProg> cs;
    for (const PlanPred &pr : q.preds) cs.push_back(pred_prog(pr));
    q.preds.clear();
    q.where = and_all(cs);
    q.compiled = true;
  }
  return any;
}

// SELECT *: the plan with every bound column projected, in binding order (names: the
// execution's columns); other plans are returned as they are
const nut_plan *expand_star(const nut_plan &p, const std::vector<std::string> &names, nut_plan &q) {
  if (!p.star) return &p;
  q = p;
  q.star = false;
  for (const std::string &nm : names) {
    int idx = -1;
    for (size_t i = 0; i < q.cols.size() && idx < 0; ++i)
      if (ieq(q.cols[i], nm)) idx = (int)i;
    if (idx < 0) {
      idx = (int)q.cols.size();
      q.cols.push_back(nm);
    }
    q.projs.push_back(idx);
    q.proj_val.emplace_back();
    q.proj_mask.emplace_back();
    PlanOut o;
    o.kind = OUT_KEY;
    o.a = (int)q.outs.size();
    o.text = o.name = nm;
    q.outs.push_back(o);
  }
  q.proj = q.projs.empty() ? -1 : q.projs[0];
  return &q;
}

// ldict / rdict (may be null): the dictionary of each column of lc / rc (typed tables)
nut_status exec_join(nut_ctx *c, const nut_plan &p, const nut_column *lc, int nl, uint64_t lrows,
                     const nut_column *rc, int nr, uint64_t rrows, uint64_t hint, nut_result *r,
                     const Dict *const *ldict, const Dict *const *rdict) {
  const size_t nc = p.cols.size();
  std::vector<int> side(nc);
  std::vector<const nut_column *> src(nc);
  std::vector<const Dict *> sdict(nc + 1, nullptr);
  auto find = [](const std::string &name, const nut_column *cols, int n) -> const nut_column * {
    for (int i = 0; i < n; ++i)
      if (cols[i].name && ieq(cols[i].name, name)) return &cols[i];
    return nullptr;
  };
  auto names = [](const std::string &q, const std::string &t, const std::string &a) {
    return ieq(q, t) || (!a.empty() && ieq(q, a));
  };
  for (size_t i = 0; i < nc; ++i) {
    const std::string &nm = p.cols[i];
    const nut_column *a = find(nm, lc, nl), *b = find(nm, rc, nr);
    const size_t dot = nm.find('.');
    if (!a && !b && dot != std::string::npos) {  // qualified: table name or alias picks the side
      const std::string q = nm.substr(0, dot), c = nm.substr(dot + 1);
      const bool l = names(q, p.table, p.talias), r = names(q, p.jtable, p.jalias);
      if (l && r) return fail(NUT_ERR_PLAN, "qualifier '" + q + "' names both tables (use aliases)");
      if (!l && !r) return fail(NUT_ERR_PLAN, "qualifier '" + q + "' names neither joined table");
      if (l) a = find(c, lc, nl);
      else b = find(c, rc, nr);
    }
    if (a && b) return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute2: column '" + nm + "' is in both tables");
    if (!a && !b) return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute2: column '" + nm + "' is not bound");
    side[i] = a ? 0 : 1;
    src[i] = a ? a : b;
    sdict[i] = a ? (ldict ? ldict[a - lc] : nullptr) : (rdict ? rdict[b - rc] : nullptr);
    if (src[i]->type != NUT_T_I64 && src[i]->type != NUT_T_F64)
      return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute2: column '" + p.cols[i] + "' has an unknown type");
    if ((a ? lrows : rrows) && !src[i]->data)
      return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute2: column '" + p.cols[i] + "' is NULL");
  }
  const int k0 = p.jkey[0], k1 = p.jkey[1];
  if (side[k0] == side[k1]) return fail(NUT_ERR_PLAN, "JOIN ON must compare a column of each table");
  const nut_column *lkey = side[k0] == 0 ? src[k0] : src[k1], *rkey = side[k0] == 0 ? src[k1] : src[k0];
  if (lkey->type != NUT_T_I64 || rkey->type != NUT_T_I64) return fail(NUT_ERR_PLAN, "JOIN keys must be int64 columns");
  if (sdict[k0] || sdict[k1])  // codes of two dictionaries do not compare
    return fail(NUT_ERR_PLAN, "JOIN keys must be integer columns (string keys are not executed)");
  // INNER builds the smaller table (decided after the pushdown below); the outer / semi /
  // anti joins preserve their side
  int ps = p.join == NUT_JOIN_INNER ? (lrows >= rrows ? 0 : 1) : (p.jright ? 1 : 0);
  const bool full = p.join == PJ_FULL;  // both tables NULL-extended; probe = the FROM table
  const bool outer = p.join == NUT_JOIN_LEFT || full;
  // what the other (build) table may feed
  int bkey = side[k0] == ps ? k1 : k0, pkey = side[k0] == ps ? k0 : k1;
  auto in_prog = [](const PProg &pp, int i) {  // (LIKE leaves read their column too)
    for (const PNode &nd : pp)
      if (reads_col(nd.op) && nd.col == i) return true;
    return false;
  };
  // read by plan q after the join: as a row decider, a projection (proj NULL: counted as a
  // row decider), or inside an aggregate
  auto reads = [&](const nut_plan &q, int ci, bool &row, bool &agg, bool *proj = nullptr) {
    bool pr = ci == q.proj;
    for (int pj : q.projs) pr = pr || pj == ci;
    for (const PProg &pp : q.proj_val) pr = pr || in_prog(pp, ci);
    for (const PProg &pp : q.proj_mask) pr = pr || in_prog(pp, ci);
    row = in_prog(q.where, ci);
    if (proj) *proj = pr;
    else row = row || pr;
    for (int k : q.keys) row = row || k == ci;
    for (const PProg &kp : q.key_progs) row = row || in_prog(kp, ci);  // computed keys
    for (const auto &sk : q.sort_keys) row = row || sk.first == ci;  // ORDER BY, projected or not
    for (const PlanPred &pr : q.preds) row = row || pr.col == ci;
    agg = false;
    for (int v : q.vals) agg = agg || v == ci;
    for (const PlanAgg &a : q.aggs) {
      for (int ref : a.refs) agg = agg || ref == ci;
      agg = agg || in_prog(a.val, ci) || in_prog(a.mask, ci);
    }
  };
  // a NULL-extended table's column may feed aggregates (they skip its NULL rows) and scan
  // projections (NULL there), not WHERE / GROUP BY / ORDER BY or IS [NOT] NULL
  auto null_side = [&](int ci) { return full || (outer && side[ci] != ps); };
  for (size_t i = 0; i < nc; ++i) {
    const int ci = (int)i;
    bool row, agg, proj;
    reads(p, ci, row, agg, &proj);
    const bool isnull = std::find(p.isnull_cols.begin(), p.isnull_cols.end(), ci) != p.isnull_cols.end();
    if (full && (row || isnull))
      return fail(NUT_ERR_PLAN, "FULL OUTER JOIN: column '" + p.cols[i] + "' may only appear inside aggregates and "
                                "projections");
    if (side[i] == ps) continue;
    if (p.join == NUT_JOIN_SEMI || p.join == NUT_JOIN_ANTI) {
      // SEMI: the other table's ON column equals the preserved one; nothing else exists
      if ((row || agg || proj) && !(p.join == NUT_JOIN_SEMI && ci == bkey))
        return fail(NUT_ERR_PLAN, "SEMI / ANTI JOIN output only the preserved table's columns ('" + p.cols[i] + "')");
    } else if (outer && (row || isnull)) {
      return fail(NUT_ERR_PLAN, "outer JOIN: the NULL-extended table's column '" + p.cols[i] +
                                    "' may only appear inside aggregates and projections" +
                                    (isnull ? " (IS [NOT] NULL over it is not executed)" : ""));
    }
  }
  // ---- predicate pushdown: WHERE conjuncts that read one table filter that table before
  // the join (nut_select_rows -> ascending row ids; the join runs on the selected keys and
  // its indices map back through the ids).  INNER: both tables; outer / semi / anti: the
  // preserved one (WHERE may not read the other table there).
  nut_plan p2 = p;
  std::vector<PProg> push[2];
  auto pushable = [&](int sd) { return sd >= 0 && !full && (p.join == NUT_JOIN_INNER || sd == ps); };
  if (p.compiled) {
    std::vector<PProg> conj, keep;
    split_and(p.where, conj);
    for (PProg &cj : conj) {
      int sd = -1;
      for (const PNode &nd : cj)
        if (reads_col(nd.op)) sd = sd < 0 || sd == side[nd.col] ? side[nd.col] : 2;
      (sd < 2 && pushable(sd) ? push[sd] : keep).push_back(std::move(cj));
    }
    p2.where = and_all(keep);
  } else {
    p2.preds.clear();
    for (const PlanPred &pr : p.preds)
      if (pushable(side[pr.col])) push[side[pr.col]].push_back(pred_prog(pr));
      else p2.preds.push_back(pr);
  }
  const nut_column *keycol[2] = {lkey, rkey};
  const int64_t *keys_s[2] = {(const int64_t *)lkey->data, (const int64_t *)rkey->data};
  uint64_t rows_s[2] = {lrows, rrows};
  DevBuf ids_s[2], keybuf[2];
  for (int sd = 0; sd < 2; ++sd) {
    if (push[sd].empty() || p.never) continue;
    nut_plan q;
    q.compiled = true;
    q.cols = p.cols;
    q.where = and_all(push[sd]);
    nut_agg_spec spec;
    ProgStore store;
    std::vector<int> agg_f64;
    nut_status es = build_spec(q, src.data(), sdict.data(), rows_s[sd], spec, store, agg_f64);
    if (es) return es;
    NUT_HIP(ids_s[sd].alloc(c, std::max<uint64_t>(rows_s[sd], 1) * 8));
    uint64_t cnt = 0;
    if (rows_s[sd]) es = nut_select_rows(c, &spec, (int64_t *)ids_s[sd].p, &cnt);
    if (es) return es;
    NUT_HIP(keybuf[sd].alloc(c, std::max<uint64_t>(cnt, 1) * 8));
    es = nut_gather_u64(c, (const uint64_t *)keycol[sd]->data, (const int64_t *)ids_s[sd].p, cnt, 0,
                        (uint64_t *)keybuf[sd].p);
    if (es) return es;
    keys_s[sd] = (const int64_t *)keybuf[sd].p;
    rows_s[sd] = cnt;
  }
  if (p.join == NUT_JOIN_INNER) ps = rows_s[0] >= rows_s[1] ? 0 : 1;
  bkey = side[k0] == ps ? k1 : k0;
  pkey = side[k0] == ps ? k0 : k1;
  const int64_t *pkd = keys_s[ps], *bkd = keys_s[1 - ps];
  const uint64_t np = rows_s[ps], nb = rows_s[1 - ps];
  std::vector<char> used(nc);  // read after the join (ON-only and pushed-down columns are not)
  for (size_t i = 0; i < nc; ++i) {
    bool row, agg;
    reads(p2, (int)i, row, agg);
    used[i] = row || agg;
  }
  // one pass into arrays of np pairs (enough unless the build keys repeat), else again
  // with the exact count; aggregates take the pairs in any order (the unordered probe)
  const int any_order = p.kind == NUT_PLAN_GROUPBY ? NUT_JOIN_ANY_ORDER : 0;
  DevBuf idx;
  uint64_t cap = std::max<uint64_t>(np, 1), npairs = 0;
  nut_status st;
  for (;;) {
    hipError_t he = idx.alloc(c, cap * 16);
    if (he != hipSuccess) return hip_fail(he, "hipMalloc (join index)");
    // the pairs carry table rows: the pushed-down selections' ids ride along as row ids
    st = join_i64_into_rows(c, bkd, (const int64_t *)ids_s[1 - ps].p, nb, pkd, (const int64_t *)ids_s[ps].p, np,
                            (full ? NUT_JOIN_LEFT : p.join) | any_order, (int64_t *)idx.p, (int64_t *)idx.p + cap, cap,
                            &npairs);
    if (st != NUT_ERR_CAPACITY || npairs <= cap) break;
    idx.reset();
    cap = npairs;
  }
  if (st) return st;
  int64_t *pi = (int64_t *)idx.p, *bi = pi + cap;
  DevBuf fidx;
  if (full) {
    // the JOIN source's rows without a match: ANTI with the roles swapped (build = the
    // FROM table's keys), appended as pairs (-1, source row)
    const uint64_t nsrc = rows_s[1 - ps];
    DevBuf anti;
    uint64_t nanti = 0;
    if (nsrc) {
      NUT_HIP(anti.alloc(c, nsrc * 16));
      st = join_i64_into_rows(c, keys_s[ps], (const int64_t *)ids_s[ps].p, rows_s[ps], keys_s[1 - ps],
                              (const int64_t *)ids_s[1 - ps].p, nsrc, NUT_JOIN_ANTI | any_order, (int64_t *)anti.p,
                              (int64_t *)anti.p + nsrc, nsrc, &nanti);
      if (st) return st;
    }
    const uint64_t tot = npairs + nanti, fcap = std::max<uint64_t>(tot, 1);
    NUT_HIP(fidx.alloc(c, fcap * 16));
    int64_t *fp = (int64_t *)fidx.p, *fb = fp + fcap;
    if (npairs) {
      NUT_HIP(hipMemcpyAsync(fp, pi, npairs * 8, hipMemcpyDeviceToDevice, c->stream));
      NUT_HIP(hipMemcpyAsync(fb, bi, npairs * 8, hipMemcpyDeviceToDevice, c->stream));
    }
    if (nanti) {
      NUT_HIP(hipMemsetAsync(fp + npairs, 0xFF, nanti * 8, c->stream));  // -1: no FROM row
      NUT_HIP(hipMemcpyAsync(fb + npairs, anti.p, nanti * 8, hipMemcpyDeviceToDevice, c->stream));
    }
    NUT_HIP(hipStreamSynchronize(c->stream));  // `anti` is freed on scope exit
    pi = fp;
    bi = fb;
    npairs = tot;
  }
  // the joined table: every plan column gathered through its side's index
  bool proj_null = false;  // a scan projecting a NULL-extended table's column
  for (size_t i = 0; i < nc && outer && p.kind != NUT_PLAN_GROUPBY; ++i) {
    bool row, agg, proj;
    reads(p2, (int)i, row, agg, &proj);
    proj_null = proj_null || (proj && null_side((int)i));
  }
  const bool mask_col = outer && (p.kind == NUT_PLAN_GROUPBY || proj_null);
  std::vector<DevBuf> bufs(nc + 1);
  std::vector<nut_column> jc(nc + 1);
  for (size_t i = 0; i < nc; ++i) {
    if (!used[i]) {  // never read: bound to its source column, not gathered
      jc[i] = nut_column{p.cols[i].c_str(), src[i]->data, src[i]->type};
      continue;
    }
    NUT_HIP(bufs[i].alloc(c, std::max<uint64_t>(npairs, 1) * 8));
    // SEMI / ANTI pairs carry no build row: the other ON column reads the preserved one
    // (outer joins: equal on matched rows; aggregates mask the NULL-extended ones)
    const bool via_probe = side[i] == ps || (p.join != NUT_JOIN_INNER && !full && (int)i == bkey);
    st = nut_gather_u64(c, (const uint64_t *)src[via_probe && (int)i == bkey ? pkey : i]->data, via_probe ? pi : bi,
                        npairs, 0, (uint64_t *)bufs[i].p);
    if (st) return st;
    jc[i] = nut_column{p.cols[i].c_str(), bufs[i].p, src[i]->type};
  }
  DevBuf lmask;
  if (mask_col) {  // aggregates over a NULL-extended table skip its NULL rows
    p2.cols.reserve(nc + 2);  // jc keeps c_str() pointers into p2.cols
    NUT_HIP(bufs[nc].alloc(c, std::max<uint64_t>(npairs, 1) * 8));
    st = join_matched(c, bi, npairs, (int64_t *)bufs[nc].p);
    if (st) return st;
    p2.cols.push_back("__matched");
    jc[nc] = nut_column{p2.cols[nc].c_str(), bufs[nc].p, NUT_T_I64};
    if (full) {  // FULL: the FROM table's columns are NULL on the source's unmatched rows
      NUT_HIP(lmask.alloc(c, std::max<uint64_t>(npairs, 1) * 8));
      st = join_matched(c, pi, npairs, (int64_t *)lmask.p);
      if (st) return st;
      p2.cols.push_back("__lmatched");
      jc.push_back(nut_column{p2.cols[nc + 1].c_str(), lmask.p, NUT_T_I64});
    }
    for (PlanAgg &a : p2.aggs) {
      bool other = false, mine = false;
      for (int ref : a.refs) {
        other = other || side[ref] != ps;
        mine = mine || side[ref] == ps;
      }
      if (other) add_null_mask(a, (int)nc);
      if (full && mine) add_null_mask(a, (int)nc + 1);
    }
    if (proj_null)
      mask_null_projections(p2, null_side, [&](int ci) { return side[ci] == ps ? (int)nc + 1 : (int)nc; });
  }
  std::vector<const nut_column *> bound(p2.cols.size());
  for (size_t i = 0; i < p2.cols.size(); ++i) bound[i] = &jc[i];
  sdict.resize(p2.cols.size());
  st = p2.kind == NUT_PLAN_GROUPBY ? exec_groupby(c, p2, bound.data(), sdict.data(), npairs, hint, r)
                                   : exec_scan(c, p2, bound.data(), sdict.data(), npairs, r);
  NUT_HIP(hipStreamSynchronize(c->stream));  // the gathered columns are freed on return
  return st;
}



// The residual step of a correlated EXISTS / NOT EXISTS: the subquery's
// rows (inner keys bk and the residual's inner column, pushed-down ids applied) are grouped
// by key with MIN and MAX of that column; each accumulated row looks its key up (a LEFT
// join on unique keys) and has a qualifying inner row iff the key is present and
//   inner <> x: min != x or max != x;  < x: min < x;  <= x: min <= x;  > x: max > x;  >= x: max >= x
// with x its outer column.  Writes the accumulated positions that pass EXISTS (or, anti,
// NOT EXISTS) to pos[0 .. *m), ascending.
nut_status residual_semi(nut_ctx *c, const nut_plan &p, int k, int op, const nut_column *icol, const nut_column *ocol,
                         const int64_t *iids, const int64_t *bk, uint64_t nb, const int64_t *pk, const int64_t *prow,
                         uint64_t np, int otab, const int64_t *oacc, bool onull, bool anti, int64_t *pos, uint64_t *m) {
  *m = 0;
  const std::string who = "subquery " + std::to_string(p.jn[k].scope);
  if (onull) return fail(NUT_ERR_PLAN, who + ": its outer column comes from a NULL-extended table");
  (void)otab;
  auto gather = [&](const void *col, const int64_t *idx, uint64_t n, uint64_t fill, DevBuf &out) -> nut_status {
    if (out.alloc(c, std::max<uint64_t>(n, 1) * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (EXISTS)");
    return n ? nut_gather_u64(c, (const uint64_t *)col, idx, n, fill, (uint64_t *)out.p) : NUT_OK;
  };
  // 1. MIN / MAX of the inner column per key of the subquery's rows
  DevBuf icb, gw;
  const void *ic = icol->data;
  nut_status st = NUT_OK;
  if (iids && (st = gather(ic, iids, nb, 0, icb))) return st;
  if (iids) ic = icb.p;
  uint64_t G = 0;
  if (nb) {
    nut_agg_spec gs;
    memset(&gs, 0, sizeof gs);
    gs.n = nb;
    gs.nkeys = 1;
    gs.keys[0] = bk;
    gs.nvals = 1;
    gs.val_col[0] = ic;
    gs.val_type[0] = icol->type;
    gs.naggs = 2;
    gs.agg_op[0] = NUT_AGG_MIN;
    gs.agg_op[1] = NUT_AGG_MAX;
    gs.agg_expr[0] = gs.agg_expr[1] = NUT_EX_COL;
    nut_groups *g = nullptr;
    st = nut_groupby(c, &gs, std::max<uint64_t>(1, std::min<uint64_t>(nb / 4, 1ull << 26)), &g);
    if (!st) st = nut_groups_size(g, &G);
    if (!st && gw.alloc(c, std::max<uint64_t>(G, 1) * 24) != hipSuccess) st = fail(NUT_ERR_OOM, "hipMalloc (EXISTS)");
    if (!st && G) st = nut_groups_to_device(g, (uint64_t *)gw.p, G);
    nut_groups_free(g);
    if (st) return st;
  }
  // 2. each accumulated row's key among the groups' (unique): (probe row, group or -1)
  DevBuf pr;
  if (pr.alloc(c, std::max<uint64_t>(np, 1) * 16) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (EXISTS)");
  int64_t *o0 = (int64_t *)pr.p, *o1 = o0 + std::max<uint64_t>(np, 1);
  uint64_t m2 = 0;
  if (np) {
    if (G) {
      st = join_i64_into_rows(c, (const int64_t *)gw.p, nullptr, G, pk, prow, np, NUT_JOIN_LEFT, o0, o1, np, &m2);
    } else {  // no inner row at all: every probe row unmatched
      st = join_i64_into_rows(c, pk, nullptr, 0, pk, prow, np, NUT_JOIN_LEFT, o0, o1, np, &m2);
    }
    if (st) return st;
    if (m2 != np) return fail(NUT_ERR_UNSUPPORTED, who + ": key lookup returned " + std::to_string(m2) + " rows");
  }
  // 3. per row: min, max (0 where unmatched) and the outer value
  DevBuf mn, mx, orow, ov;
  if (G && ((st = gather((const uint64_t *)gw.p + G, o1, np, 0, mn)) || (st = gather((const uint64_t *)gw.p + 2 * G, o1, np, 0, mx))))
    return st;
  if (!G && (mn.alloc(c, std::max<uint64_t>(np, 1) * 8) != hipSuccess || mx.alloc(c, std::max<uint64_t>(np, 1) * 8) != hipSuccess))
    return fail(NUT_ERR_OOM, "hipMalloc (EXISTS)");
  const int64_t *orows = o0;  // accumulated position -> the outer table's row
  if (oacc) {
    if ((st = gather(oacc, o0, np, ~0ull, orow))) return st;
    orows = (const int64_t *)orow.p;
  }
  if ((st = gather(ocol->data, orows, np, 0, ov))) return st;
  // 4. the rows that pass: SEMI (g >= 0) and cond; ANTI its negation
  nut_plan q;
  q.compiled = true;
  q.cols = {"__g", "__mn", "__mx", "__x"};
  auto col = [](PProg &pp, int ci) {
    PNode n;
    n.op = NUT_P_COL;
    n.col = ci;
    pp.push_back(n);
  };
  PProg &w = q.where;
  col(w, 0);
  emit_int(w, 0);
  emit(w, NUT_P_GE);
  if (op == NUT_P_NE) {
    col(w, 1), col(w, 3), emit(w, NUT_P_NE);
    col(w, 2), col(w, 3), emit(w, NUT_P_NE);
    emit(w, NUT_P_OR);
  } else {
    col(w, op == NUT_P_LT || op == NUT_P_LE ? 1 : 2), col(w, 3), emit(w, op);
  }
  emit(w, NUT_P_AND);
  if (anti) emit(w, NUT_P_NOT);
  const nut_column qc[4] = {{q.cols[0].c_str(), o1, NUT_T_I64},
                            {q.cols[1].c_str(), mn.p, icol->type},
                            {q.cols[2].c_str(), mx.p, icol->type},
                            {q.cols[3].c_str(), ov.p, ocol->type}};
  const nut_column *qb[4] = {&qc[0], &qc[1], &qc[2], &qc[3]};
  const Dict *qd[4] = {nullptr, nullptr, nullptr, nullptr};
  nut_agg_spec spec;
  ProgStore store;
  std::vector<int> agg_f64;
  if ((st = build_spec(q, qb, qd, np, spec, store, agg_f64))) return st;
  DevBuf sel;
  if (sel.alloc(c, std::max<uint64_t>(np, 1) * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (EXISTS)");
  uint64_t ns = 0;
  if (np && (st = nut_select_rows(c, &spec, (int64_t *)sel.p, &ns))) return st;
  // 5. their accumulated positions (the probe rows of step 2, in probe order)
  if (ns && (st = nut_gather_u64(c, (const uint64_t *)o0, (const int64_t *)sel.p, ns, 0, (uint64_t *)pos))) return st;
  NUT_HIP(hipStreamSynchronize(c->stream));
  *m = ns;
  return NUT_OK;
}

// A chain of INNER joins (nut_plan_executen): FROM t0 JOIN t1 ON .. JOIN t2 ON ..  Single-
// table WHERE conjuncts are pushed down per table; the accumulated join result is kept as
// one row-id array per joined table (the probe side); each step builds on the next table.
// tdicts (typed tables, nut_table_executen): per table, the dictionary of each column
// (NULL = numeric); string columns filter, group and project with their own table's codes.
nut_status exec_joinn(nut_ctx *c, const nut_plan &p, const nut_column *const *tabs, const int *ncols,
                      const uint64_t *nrows, int nt, uint64_t hint, nut_result *r,
                      const Dict *const *const *tdicts) {
  const size_t nc = p.cols.size();
  if (nt != (int)p.jn.size() + 1)
    return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: the plan joins " + std::to_string(p.jn.size() + 1) +
                                         " tables, got " + std::to_string(nt));
  std::vector<std::string> tname(nt), talias(nt);
  tname[0] = p.table;
  talias[0] = p.talias;
  for (int k = 1; k < nt; ++k) tname[k] = p.jn[k - 1].table, talias[k] = p.jn[k - 1].alias;
  auto find = [&](const std::string &name, int t) -> const nut_column * {
    for (int i = 0; i < ncols[t]; ++i)
      if (tabs[t][i].name && ieq(tabs[t][i].name, name)) return &tabs[t][i];
    return nullptr;
  };
  // scopes: the FROM table and JOIN sources are the outer query's (0); an EXISTS / IN
  // step's table is its subquery's.  An unqualified name of scope s >= 1 binds to scope s's
  // table if it has the column, else to the outer tables (a correlation); a scope-0 name
  // to the outer tables only.  Qualified names bind by qualifier whatever their scope.
  std::vector<int> tscope(nt, 0);
  for (int k = 1; k < nt; ++k) tscope[k] = p.jn[k - 1].scope;
  std::vector<int> side(nc);
  std::vector<const nut_column *> src(nc);
  std::vector<const Dict *> sdict(nc + 1, nullptr);
  for (size_t i = 0; i < nc; ++i) {
    std::string nm;
    const int sc = name_scope(p.cols[i], &nm);
    int hit = -1, nh = 0;
    for (int t = 0; t < nt && sc > 0 && !nh; ++t)
      if (tscope[t] == sc && find(nm, t)) hit = t, ++nh;
    for (int t = 0; t < nt && !nh; ++t)
      if (tscope[t] == 0 && find(nm, t)) hit = t, ++nh;
    for (int t = hit + 1; t < nt && nh; ++t)
      if (tscope[t] == 0 && tscope[hit] == 0 && find(nm, t)) ++nh;
    const nut_column *col = hit >= 0 ? find(nm, hit) : nullptr;
    const size_t dot = nm.find('.');
    if (!nh && dot != std::string::npos) {
      const std::string q = nm.substr(0, dot), cn = nm.substr(dot + 1);
      for (int t = 0; t < nt; ++t)
        if (ieq(q, tname[t]) || (!talias[t].empty() && ieq(q, talias[t]))) hit = t, ++nh;
      if (nh > 1) return fail(NUT_ERR_PLAN, "qualifier '" + q + "' names several tables (use aliases)");
      if (nh == 0) return fail(NUT_ERR_PLAN, "qualifier '" + q + "' names no joined table");
      col = find(cn, hit);
      if (!col) nh = 0;
    }
    if (nh > 1) return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: column '" + nm + "' is in several tables");
    if (!col) return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: column '" + nm + "' is not bound");
    if (sc > 0 && tscope[hit] != 0 && tscope[hit] != sc)
      return fail(NUT_ERR_PLAN, "a subquery reads column '" + nm + "' of another subquery's table");
    if (col->type != NUT_T_I64 && col->type != NUT_T_F64)
      return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: column '" + nm + "' has an unknown type");
    if (nrows[hit] && !col->data) return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: column '" + nm + "' is NULL");
    side[i] = hit;
    src[i] = col;
    if (tdicts && tdicts[hit]) sdict[i] = tdicts[hit][col - tabs[hit]];
  }
  // EXISTS / IN steps: each conjunct of the subquery's WHERE is a filter of its own table
  // (pushed down), the correlation equality (EXISTS: the first equality of a column of
  // its table with an earlier table's int64 column is the key) or the residual: one
  // comparison `inner <op> outer` (executed through MIN / MAX per key, below)
  std::vector<std::array<int, 2>> jkey(nt - 1);
  std::vector<std::vector<PProg>> sub_push(nt);
  struct Residual {
    int op = -1, in = -1, out = -1;  // inner <op> outer
  };
  std::vector<Residual> res(nt - 1);
  for (int k = 0; k + 1 < nt; ++k) {
    const nut_plan::JoinStep &js = p.jn[k];
    const int t = k + 1;
    jkey[k] = {js.key[0], js.key[1]};
    std::vector<PProg> conj;
    split_and(js.cond, conj);
    if (!js.scope) {  // ON filters: conditions on the step's own table, applied before it joins
      for (PProg &cj : conj) {
        for (const PNode &nd : cj)
          if (reads_col(nd.op) && side[nd.col] != t)
            return fail(NUT_ERR_PLAN, "JOIN " + std::to_string(t) + ": an ON condition beyond the key equality must read '" +
                                          tname[t] + "' alone (column '" + p.cols[nd.col] + "')");
        sub_push[t].push_back(std::move(cj));
      }
      continue;
    }
    for (PProg &cj : conj) {
      bool inner = false, outer = false, later = false;
      for (const PNode &nd : cj)
        if (reads_col(nd.op)) {
          inner = inner || side[nd.col] == t;
          outer = outer || side[nd.col] < t;
          later = later || side[nd.col] > t;
        }
      if (later) return fail(NUT_ERR_PLAN, "subquery " + std::to_string(js.scope) + ": reads a later table");
      if (!outer) {  // a filter of the subquery's own table (or a constant)
        sub_push[t].push_back(std::move(cj));
        continue;
      }
      if (!inner)
        return fail(NUT_ERR_PLAN, "subquery " + std::to_string(js.scope) +
                                      ": a condition on the outer query's tables alone is not executed inside EXISTS / IN");
      const bool cmp2 = cj.size() == 3 && cj[0].op == NUT_P_COL && cj[1].op == NUT_P_COL && cj[2].op >= NUT_P_LT &&
                        cj[2].op <= NUT_P_NE;
      if (!cmp2)
        return fail(NUT_ERR_PLAN, "subquery " + std::to_string(js.scope) +
                                      ": a correlated condition must compare a column of its table with an outer column");
      int a = cj[0].col, b = cj[1].col, op = cj[2].op;
      if (side[a] != t) {  // inner on the left: a <op> b
        std::swap(a, b);
        op = op == NUT_P_LT ? NUT_P_GT : op == NUT_P_GT ? NUT_P_LT : op == NUT_P_LE ? NUT_P_GE : op == NUT_P_GE ? NUT_P_LE : op;
      }
      if (op == NUT_P_EQ && jkey[k][0] < 0 && src[a]->type == NUT_T_I64 && src[b]->type == NUT_T_I64) {
        jkey[k] = {b, a};
      } else if (res[k].op < 0 && op != NUT_P_EQ) {
        res[k] = Residual{op, a, b};
      } else {
        return fail(NUT_ERR_PLAN, "subquery " + std::to_string(js.scope) +
                                      ": one equality with the outer query and at most one other comparison are executed");
      }
    }
    if (jkey[k][0] < 0)
      return fail(NUT_ERR_PLAN, "EXISTS: the subquery needs an equality between an int64 column of its table and one of "
                                "the outer query's (an uncorrelated EXISTS is not executed)");
  }
  std::vector<int> knew(nt - 1), kold(nt - 1);
  for (int k = 0; k + 1 < nt; ++k) {
    const int a = jkey[k][0], b = jkey[k][1], t = k + 1;
    if (side[a] == t && side[b] < t) knew[k] = a, kold[k] = b;
    else if (side[b] == t && side[a] < t) knew[k] = b, kold[k] = a;
    else return fail(NUT_ERR_PLAN, "JOIN " + std::to_string(t) + ": ON must compare a column of '" + tname[t] +
                                       "' with a column of an earlier table");
    if (src[a]->type != NUT_T_I64 || src[b]->type != NUT_T_I64) return fail(NUT_ERR_PLAN, "JOIN keys must be int64 columns");
    if (sdict[a] || sdict[b])  // codes of two dictionaries do not compare
      return fail(NUT_ERR_PLAN, "JOIN " + std::to_string(t) + ": string keys are not executed (each table has its own "
                                    "dictionary)");
  }
  auto in_prog = [](const PProg &pp, int i) {
    for (const PNode &nd : pp)
      if (reads_col(nd.op) && nd.col == i) return true;
    return false;
  };
  // read by plan q after the joins: as a row decider / key, a projection, or inside an aggregate
  auto reads = [&](const nut_plan &q, int ci, bool &row, bool &agg, bool &proj) {
    proj = ci == q.proj;
    for (int pj : q.projs) proj = proj || pj == ci;
    for (const PProg &pp : q.proj_val) proj = proj || in_prog(pp, ci);
    for (const PProg &pp : q.proj_mask) proj = proj || in_prog(pp, ci);
    row = in_prog(q.where, ci);
    for (int k2 : q.keys) row = row || k2 == ci;
    for (const PProg &kp : q.key_progs) row = row || in_prog(kp, ci);  // computed keys
    for (const auto &sk : q.sort_keys) row = row || sk.first == ci;  // ORDER BY, projected or not
    for (const PlanPred &pr : q.preds) row = row || pr.col == ci;
    agg = false;
    for (int v : q.vals) agg = agg || v == ci;
    for (const PlanAgg &a : q.aggs) {
      for (int ref : a.refs) agg = agg || ref == ci;
      agg = agg || in_prog(a.val, ci) || in_prog(a.mask, ci);
    }
  };
  // NULL-extended tables: the one a LEFT step joins, every earlier one after a RIGHT step,
  // both sides of a FULL step (their accumulated row ids hold -1 on the NULL rows; a later
  // step's ON key from such a table matches nothing there).  Their columns may only feed
  // aggregates, which skip the NULL rows, and projections (NULL there).  A LEFT SEMI / ANTI
  // step's table only filters: its columns are not output.
  std::vector<char> nullable(nt, 0), absent(nt, 0);
  for (int k = 0; k + 1 < nt; ++k) {
    const int t = k + 1, type = p.jn[k].type;
    if (type == NUT_JOIN_LEFT || type == PJ_FULL) nullable[t] = 1;
    if (type == PJ_RIGHT || type == PJ_FULL)
      for (int v = 0; v < t; ++v) nullable[v] = 1;
    if (type == NUT_JOIN_SEMI || type == NUT_JOIN_ANTI) absent[t] = 1;
    if (absent[side[kold[k]]])
      return fail(NUT_ERR_PLAN, "JOIN " + std::to_string(t) + ": ON reads a SEMI / ANTI-joined table ('" +
                                    tname[side[kold[k]]] + "'), whose columns are not output");
  }
  bool proj_null = false;  // a scan projecting a NULL-extended table's column (NULL there)
  for (size_t i = 0; i < nc; ++i) {
    bool row, agg, proj;
    reads(p, (int)i, row, agg, proj);
    const bool isnull = std::find(p.isnull_cols.begin(), p.isnull_cols.end(), (int)i) != p.isnull_cols.end();
    if ((row || agg || proj) && absent[side[i]])
      return fail(NUT_ERR_PLAN, "SEMI / ANTI JOIN: the columns of '" + tname[side[i]] + "' are not output ('" +
                                    p.cols[i] + "')");
    if ((row || isnull) && nullable[side[i]])
      return fail(NUT_ERR_PLAN, "outer JOIN: the NULL-extended table's column '" + p.cols[i] +
                                    "' may only appear inside aggregates and projections" +
                                    (isnull ? " (IS [NOT] NULL over it is not executed)" : ""));
    proj_null = proj_null || (proj && nullable[side[i]] && p.kind != NUT_PLAN_GROUPBY);
  }
  nut_plan p2 = p;
  std::vector<std::vector<PProg>> push(nt);
  if (p.compiled) {
    std::vector<PProg> conj, keep;
    split_and(p.where, conj);
    for (PProg &cj : conj) {
      int sd = -1;
      for (const PNode &nd : cj)
        if (reads_col(nd.op)) sd = sd < 0 || sd == side[nd.col] ? side[nd.col] : nt;
      (sd >= 0 && sd < nt ? push[sd] : keep).push_back(std::move(cj));
    }
    p2.where = and_all(keep);
  } else {
    p2.preds.clear();
    for (const PlanPred &pr : p.preds) push[side[pr.col]].push_back(pred_prog(pr));
  }
  for (int t = 0; t < nt; ++t)
    for (PProg &cj : sub_push[t]) push[t].push_back(std::move(cj));
  std::vector<DevBuf> ids(nt);
  std::vector<uint64_t> rows(nrows, nrows + nt);
  for (int t = 0; t < nt; ++t) {
    if (push[t].empty() || p.never) continue;
    nut_plan q;
    q.compiled = true;
    q.cols = p.cols;
    q.where = and_all(push[t]);
    nut_agg_spec spec;
    ProgStore store;
    std::vector<int> agg_f64;
    nut_status es = build_spec(q, src.data(), sdict.data(), rows[t], spec, store, agg_f64);
    if (es) return es;
    NUT_HIP(ids[t].alloc(c, std::max<uint64_t>(rows[t], 1) * 8));
    uint64_t cnt = 0;
    if (rows[t]) es = nut_select_rows(c, &spec, (int64_t *)ids[t].p, &cnt);
    if (es) return es;
    rows[t] = cnt;
  }
  auto gather_to = [&](const void *col, const int64_t *idx, uint64_t n, DevBuf &out) -> nut_status {
    if (out.alloc(c, std::max<uint64_t>(n, 1) * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (join)");
    return n ? nut_gather_u64(c, (const uint64_t *)col, idx, n, 0, (uint64_t *)out.p) : NUT_OK;
  };
  // accumulated row ids through positions (a -1 position, RIGHT / FULL: row id -1)
  auto gather_rows = [&](const int64_t *ids_, const int64_t *idx, uint64_t n, DevBuf &out) -> nut_status {
    if (out.alloc(c, std::max<uint64_t>(n, 1) * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (join)");
    return n ? nut_gather_u64(c, (const uint64_t *)ids_, idx, n, ~0ull, (uint64_t *)out.p) : NUT_OK;
  };
  // positions i < n with (rowids[i] cmp 0), ascending (a one-column WHERE program)
  auto select_pos = [&](const int64_t *rowids, uint64_t n, int cmp, DevBuf &out, uint64_t *cnt) -> nut_status {
    nut_plan q;
    q.compiled = true;
    q.cols = {"__row"};
    PNode col;
    col.op = NUT_P_COL;
    col.col = 0;
    q.where.push_back(col);
    emit_int(q.where, 0);
    emit(q.where, cmp);
    const nut_column rc{q.cols[0].c_str(), rowids, NUT_T_I64};
    const nut_column *rs[1] = {&rc};
    const Dict *rd[1] = {nullptr};
    nut_agg_spec spec;
    ProgStore store;
    std::vector<int> agg_f64;
    nut_status es = build_spec(q, rs, rd, n, spec, store, agg_f64);
    if (es) return es;
    if (out.alloc(c, std::max<uint64_t>(n, 1) * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (join)");
    *cnt = 0;
    return n ? nut_select_rows(c, &spec, (int64_t *)out.p, cnt) : NUT_OK;
  };
  std::vector<DevBuf> acc(nt);
  std::vector<const int64_t *> accp(nt, nullptr);
  accp[0] = (const int64_t *)ids[0].p;
  uint64_t ncur = rows[0];
  nut_status st = NUT_OK;
  std::vector<char> cur_null(nt, 0);  // table v's accumulated row ids may hold -1 (so far)
  const int any = p.kind == NUT_PLAN_GROUPBY ? NUT_JOIN_ANY_ORDER : 0;
  for (int k = 0; k + 1 < nt && !st; ++k) {
    const int t = k + 1, u = side[kold[k]], type = p.jn[k].type;
    // accumulated positions without a match stay (their table-t row -1)
    const bool keep = type == NUT_JOIN_LEFT || type == PJ_FULL || type == NUT_JOIN_ANTI;
    DevBuf pk, bk, vpos, vrow, npos;
    const int64_t *pkd = (const int64_t *)src[kold[k]]->data, *bkd = (const int64_t *)src[knew[k]]->data;
    const int64_t *prow = nullptr;  // position of each accumulated key (nullptr: its index)
    uint64_t np = ncur, nnull = 0;
    if (cur_null[u]) {
      // a NULL ON key matches nothing: only the positions whose table-u row exists take
      // part; LEFT / FULL / ANTI append the others as (position, -1)
      if ((st = select_pos(accp[u], ncur, NUT_P_GE, vpos, &np))) break;
      if (keep && (st = select_pos(accp[u], ncur, NUT_P_LT, npos, &nnull))) break;
      if ((st = gather_to(accp[u], (const int64_t *)vpos.p, np, vrow))) break;
      if ((st = gather_to(pkd, (const int64_t *)vrow.p, np, pk))) break;
      pkd = (const int64_t *)pk.p;
      prow = (const int64_t *)vpos.p;
    } else if (accp[u]) {
      if ((st = gather_to(pkd, accp[u], ncur, pk))) break;
      pkd = (const int64_t *)pk.p;
    }
    if (ids[t].p) {
      if ((st = gather_to(bkd, (const int64_t *)ids[t].p, rows[t], bk))) break;
      bkd = (const int64_t *)bk.p;
    }
    // pairs (accumulated position, table-t row), -1 = none; the pushed-down ids ride along
    // as rows.  RIGHT probes with table t (its rows all stay) against the accumulated keys.
    const bool right = type == PJ_RIGHT;
    DevBuf pairs;
    uint64_t cap = std::max<uint64_t>(right ? rows[t] : np, 1), m = 0, half = 0;
    const uint64_t extra = nnull + (type == PJ_FULL ? rows[t] : 0);  // appended below
    if (res[k].op >= 0) {  // EXISTS / NOT EXISTS with a residual comparison: positions kept
      half = cap + extra;
      if (pairs.alloc(c, half * 16) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (join index)");
      st = residual_semi(c, p, k, res[k].op, src[res[k].in], src[res[k].out], ids[t].p ? (const int64_t *)ids[t].p : nullptr,
                         bkd, rows[t], pkd, prow, np, side[res[k].out], accp[side[res[k].out]], cur_null[side[res[k].out]],
                         type == NUT_JOIN_ANTI, (int64_t *)pairs.p, &m);
      if (st) break;
    }
    for (; res[k].op < 0;) {
      half = cap + extra;
      if (pairs.alloc(c, half * 16) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (join index)");
      int64_t *o0 = (int64_t *)pairs.p, *o1 = o0 + half;
      if (right)  // probe = table t: (t row, position)
        st = join_i64_into_rows(c, pkd, prow, np, bkd, (const int64_t *)ids[t].p, rows[t], NUT_JOIN_LEFT | any, o1, o0,
                                cap, &m);
      else
        st = join_i64_into_rows(c, bkd, (const int64_t *)ids[t].p, rows[t], pkd, prow, np,
                                (type == PJ_FULL ? NUT_JOIN_LEFT : type) | any, o0, o1, cap, &m);
      if (st != NUT_ERR_CAPACITY || m <= cap) break;
      pairs.reset();
      cap = m;
    }
    if (st) break;
    int64_t *pi = (int64_t *)pairs.p, *bi = pi + half;
    if (nnull) {
      NUT_HIP(hipMemcpyAsync(pi + m, npos.p, nnull * 8, hipMemcpyDeviceToDevice, c->stream));
      NUT_HIP(hipMemsetAsync(bi + m, 0xFF, nnull * 8, c->stream));  // -1: no table-t row
      m += nnull;
    }
    if (type == PJ_FULL && rows[t]) {
      // table t's rows without a match: ANTI with the roles swapped, appended as (-1, row)
      uint64_t na = 0;
      st = join_i64_into_rows(c, pkd, prow, np, bkd, (const int64_t *)ids[t].p, rows[t], NUT_JOIN_ANTI | any,
                              bi + m, pi + m, rows[t], &na);
      if (st) break;
      NUT_HIP(hipMemsetAsync(pi + m, 0xFF, na * 8, c->stream));  // -1: no accumulated row
      m += na;
    }
    const bool semi = type == NUT_JOIN_SEMI || type == NUT_JOIN_ANTI;  // table t contributes no rows
    std::vector<DevBuf> next(nt);
    for (int v = 0; v <= t && !st; ++v) {
      if (v == t && semi) continue;
      if (v < t && accp[v]) {
        st = gather_rows(accp[v], pi, m, next[v]);
      } else {
        if (next[v].alloc(c, std::max<uint64_t>(m, 1) * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc");
        if (m) NUT_HIP(hipMemcpyAsync(next[v].p, v == t ? bi : pi, m * 8, hipMemcpyDeviceToDevice, c->stream));
      }
    }
    if (st) break;
    NUT_HIP(hipStreamSynchronize(c->stream));
    for (int v = 0; v <= t; ++v) {
      if (v == t && semi) continue;
      std::swap(acc[v].p, next[v].p);
      std::swap(acc[v].s, next[v].s);
      accp[v] = (const int64_t *)acc[v].p;
    }
    ncur = m;
    if (type == NUT_JOIN_LEFT || type == PJ_FULL) cur_null[t] = 1;
    if (type == PJ_RIGHT || type == PJ_FULL)
      for (int v = 0; v < t; ++v) cur_null[v] = 1;
  }
  if (st) return st;
  std::vector<DevBuf> bufs(nc);
  std::vector<nut_column> jc(nc);
  for (size_t i = 0; i < nc; ++i) {
    const int ci = (int)i;
    bool used = ci == p2.proj || in_prog(p2.where, ci);
    for (int pj : p2.projs) used = used || pj == ci;
    for (const PProg &pp : p2.proj_val) used = used || in_prog(pp, ci);
    for (const PProg &pp : p2.proj_mask) used = used || in_prog(pp, ci);
    for (int k2 : p2.keys) used = used || k2 == ci;
    for (const PProg &kp : p2.key_progs) used = used || in_prog(kp, ci);  // computed GROUP BY keys
    for (const auto &sk : p2.sort_keys) used = used || sk.first == ci;
    for (const PlanPred &pr : p2.preds) used = used || pr.col == ci;
    for (int v : p2.vals) used = used || v == ci;
    for (const PlanAgg &a : p2.aggs) {
      for (int ref : a.refs) used = used || ref == ci;
      used = used || in_prog(a.val, ci) || in_prog(a.mask, ci);
    }
    if (!used || !accp[side[i]]) {
      jc[i] = nut_column{p.cols[i].c_str(), src[i]->data, src[i]->type};
      continue;
    }
    st = gather_to(src[i]->data, accp[side[i]], ncur, bufs[i]);
    if (st) return st;
    jc[i] = nut_column{p.cols[i].c_str(), bufs[i].p, src[i]->type};
  }
  // aggregates over a NULL-extended table skip its NULL rows: (__matched<t> != 0) per table read
  std::vector<DevBuf> mbuf(nt);
  p2.cols.reserve(nc + nt);  // jc keeps c_str() pointers into p2.cols
  std::vector<int> mflag(nt, -1);
  for (int v = 0; v < nt && (p2.kind == NUT_PLAN_GROUPBY || proj_null); ++v) {
    if (!nullable[v]) continue;  // (table 0 too, after a RIGHT / FULL step)
    std::vector<PlanAgg *> reading;
    for (PlanAgg &a : p2.aggs) {
      bool rd = false;
      for (int ref : a.refs) rd = rd || side[ref] == v;
      if (rd) reading.push_back(&a);
    }
    bool projected = false;
    for (size_t i = 0; i < nc && proj_null; ++i) {
      bool row, agg, proj;
      reads(p2, (int)i, row, agg, proj);
      projected = projected || (proj && side[i] == v);
    }
    if (reading.empty() && !projected) continue;
    if (mbuf[v].alloc(c, std::max<uint64_t>(ncur, 1) * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc");
    if ((st = join_matched(c, accp[v], ncur, (int64_t *)mbuf[v].p))) return st;
    const int mc = (int)p2.cols.size();
    p2.cols.push_back("__matched" + std::to_string(v));
    jc.push_back(nut_column{p2.cols[mc].c_str(), mbuf[v].p, NUT_T_I64});
    for (PlanAgg *a : reading) add_null_mask(*a, mc);
    mflag[v] = mc;
  }
  if (proj_null)
    mask_null_projections(p2, [&](int ci) { return ci < (int)nc && nullable[side[ci]] != 0; },
                          [&](int ci) { return mflag[side[ci]]; });
  sdict.resize(p2.cols.size());
  std::vector<const nut_column *> bound(jc.size());
  for (size_t i = 0; i < jc.size(); ++i) bound[i] = &jc[i];
  st = p2.kind == NUT_PLAN_GROUPBY ? exec_groupby(c, p2, bound.data(), sdict.data(), ncur, hint, r)
                                   : exec_scan(c, p2, bound.data(), sdict.data(), ncur, r);
  NUT_HIP(hipStreamSynchronize(c->stream));
  return st;
}


nut_status stage_host(nut_ctx *c, const nut_column *cols, int n, uint64_t rows, HostStage &hs, const nut_column **out) {
  *out = cols;
  bool any = false;
  for (int i = 0; i < n; ++i) any = any || (cols[i].type & NUT_COL_HOST);
  if (!any) return NUT_OK;
  hs.cols.assign(cols, cols + n);
  for (nut_column &col : hs.cols) {
    if (!(col.type & NUT_COL_HOST)) continue;
    col.type &= ~NUT_COL_HOST;
    if (!rows || !col.data) continue;
    hs.bufs.emplace_back();
    NUT_HIP(hs.bufs.back().alloc(c, rows * 8));
    NUT_HIP(hipMemcpyAsync(hs.bufs.back().p, col.data, rows * 8, hipMemcpyHostToDevice, c->stream));
    col.data = hs.bufs.back().p;
  }
  *out = hs.cols.data();
  return NUT_OK;
}


}  // namespace plan
}  // namespace nut
