// sql_exec_groupby.cpp — executing GROUPBY plans: packed key programs (up to 8 keys),
// countUnique, HAVING / ORDER BY / LIMIT and arithmetic over the group result.
#include "sql_plan.hpp"

namespace nut {
namespace plan {

// ---- GROUP BY over key programs: computed keys, up to kMaxGroupKeys
// keys, countUnique.  The group-by kernels take two 64-bit key words, so the key tuple is
// packed: one range pass (MIN / MAX of every key program under WHERE) sizes each key's
// field, keys are laid out in order from the top bit of word 0 (63 bits per word; a key
// whose range needs 64 bits takes a word of its own, raw), and each word is a program
// OR-ing (key - min) << shift — evaluated inside the same streaming kernel.  The packing is
// order-preserving, so groups still arrive sorted by key tuple.  countUnique(x) adds x as a
// last field: GROUP BY (keys, x), then a count per key-word tuple over those groups.
struct KeyField {
  nut_prog prog{0, nullptr};
  int64_t mn = 0;
  int bits = 64;  // 64: raw, a word of its own
  int word = 0, shift = 0;
};

// place fields [0, f.size()) greedily; false if they need more than two words
bool layout_fields(std::vector<KeyField> &f, int *nwords) {
  int w = 0, used = 0;
  for (KeyField &k : f) {
    if (k.bits >= 64) {
      if (used) ++w;
      k.word = w;
      k.shift = 0;
      used = 64;
    } else {
      if (used + k.bits > 63) ++w, used = 0;
      k.word = w;
      k.shift = 63 - used - k.bits;
      used += k.bits;
    }
    if (w >= NUT_MAX_KEYS) return false;
  }
  *nwords = f.empty() ? 0 : w + 1;
  return true;
}

// the program of key word w: OR over its fields of (prog - mn) << shift (raw: prog);
// `drop` >= 0: leave field `drop` out
nut_status word_prog(const std::vector<KeyField> &f, int w, int drop, ProgStore &store, nut_prog &out) {
  store.nodes.emplace_back();
  std::vector<nut_prog_node> &v = store.nodes.back();
  int terms = 0;
  for (size_t j = 0; j < f.size(); ++j) {
    const KeyField &k = f[j];
    if (k.word != w || (int)j == drop) continue;
    v.insert(v.end(), k.prog.node, k.prog.node + k.prog.n);
    if (k.bits < 64) {
      if (k.mn) {
        v.push_back(nut_prog_node{NUT_P_I64, 0, k.mn});
        v.push_back(nut_prog_node{NUT_P_SUB, 0, 0});
      }
      if (k.shift) {
        v.push_back(nut_prog_node{NUT_P_I64, 0, k.shift});
        v.push_back(nut_prog_node{NUT_P_SHL, 0, 0});
      }
    }
    if (terms++) v.push_back(nut_prog_node{NUT_P_BITOR, 0, 0});
  }
  if (!terms) v.push_back(nut_prog_node{NUT_P_I64, 0, 0});
  if (v.size() > NUT_MAX_PROG_NODES)
    return fail(NUT_ERR_PLAN, "GROUP BY keys: the packed key word program exceeds 256 nodes");
  out.n = (int32_t)v.size();
  out.node = v.data();
  return NUT_OK;
}

// AND of two programs (either may be empty)
nut_prog and_prog(const nut_prog &a, const nut_prog &b, ProgStore &store) {
  if (!a.n) return b;
  if (!b.n) return a;
  store.nodes.emplace_back(a.node, a.node + a.n);
  std::vector<nut_prog_node> &v = store.nodes.back();
  v.insert(v.end(), b.node, b.node + b.n);
  v.push_back(nut_prog_node{NUT_P_AND, 0, 0});
  return nut_prog{(int32_t)v.size(), v.data()};
}

// run a group-by and copy its groups to the host (keys [ng x nk], words [ng x na])
nut_status run_groupby(nut_ctx *c, const nut_agg_spec &s, uint64_t hint, std::vector<int64_t> &keys,
                       std::vector<uint64_t> &words, uint64_t &ng) {
  nut_groups *g = nullptr;
  nut_status st = nut_groupby(c, &s, hint, &g);
  if (st) return st;
  st = nut_groups_size(g, &ng);
  if (!st) {
    keys.assign(ng * std::max(s.nkeys, 1) + 1, 0);
    words.assign(ng * std::max(s.naggs, 1) + 1, 0);
    st = nut_groups_to_host(g, keys.data(), words.data(), ng);
  }
  nut_groups_free(g);
  return st;
}

nut_status groupby_packed(nut_ctx *c, const nut_plan &p, const nut_agg_spec &s, const GbExtra &gx, ProgStore &store,
                          uint64_t hint, std::vector<int64_t> &keys, std::vector<uint64_t> &words, uint64_t &ng) {
  const size_t nkey = gx.key.size(), na = p.aggs.size();
  ng = 0;
  keys.assign(1, 0);
  words.assign(1, 0);
  if (!s.n) return NUT_OK;  // no rows: no groups
  std::vector<int> cus;  // countUnique aggregates
  for (size_t a = 0; a < na; ++a)
    if (p.aggs[a].distinct) cus.push_back((int)a);
  // fields: the keys, then each countUnique argument
  std::vector<KeyField> fk(nkey);
  for (size_t j = 0; j < nkey; ++j) fk[j].prog = gx.key[j];
  std::vector<KeyField> fx(cus.size());
  for (size_t i = 0; i < cus.size(); ++i) fx[i].prog = gx.cu_val[cus[i]];
  ng = 0;
  const bool ranges = nkey > NUT_MAX_KEYS || !cus.empty();
  if (ranges && s.n) {
    // MIN / MAX of every field under WHERE (a countUnique argument under its mask too)
    std::vector<std::pair<KeyField *, nut_prog>> all;
    for (KeyField &k : fk) all.push_back({&k, nut_prog{0, nullptr}});
    for (size_t i = 0; i < cus.size(); ++i) all.push_back({&fx[i], gx.cu_mask[cus[i]]});
    for (size_t b = 0; b < all.size(); b += NUT_MAX_AGGS / 2) {
      nut_agg_spec r = s;
      r.nkeys = 0;
      r.naggs = 0;
      for (size_t j = b; j < all.size() && j < b + NUT_MAX_AGGS / 2; ++j)
        for (int op : {NUT_AGG_MIN, NUT_AGG_MAX}) {
          r.agg_op[r.naggs] = op;
          r.agg_val[r.naggs] = all[j].first->prog;
          r.agg_mask[r.naggs] = all[j].second;
          r.naggs++;
        }
      std::vector<int64_t> rk;
      std::vector<uint64_t> rw;
      uint64_t rg = 0;
      nut_status st = run_groupby(c, r, 1, rk, rw, rg);
      if (st) return st;
      if (rg == 0) return NUT_OK;  // no row passes WHERE: no groups
      for (size_t j = b; j < all.size() && j < b + NUT_MAX_AGGS / 2; ++j) {
        const int64_t mn = (int64_t)rw[2 * (j - b)], mx = (int64_t)rw[2 * (j - b) + 1];
        KeyField &k = *all[j].first;
        if (mx < mn) {  // a masked argument that took no row
          k.mn = 0;
          k.bits = 0;
          continue;
        }
        const uint64_t range = (uint64_t)mx - (uint64_t)mn;
        k.mn = mn;
        k.bits = range ? 64 - __builtin_clzll(range) : 0;
      }
    }
  }
  int nwk = 0;
  if (!layout_fields(fk, &nwk))
    return fail(NUT_ERR_UNSUPPORTED, "GROUP BY keys: their value ranges need more than 2 x 63 bits packed (" +
                                         std::to_string(nkey) + " keys)");
  // main pass: the keys as packed words, the plan's other aggregates
  nut_agg_spec m = s;
  m.nkeys = nwk;
  for (int w = 0; w < nwk; ++w) {
    nut_status st = word_prog(fk, w, -1, store, m.key_prog[w]);
    if (st) return st;
  }
  const bool dummy = m.naggs == 0;  // (only countUnique aggregates: a COUNT enumerates groups)
  if (dummy) {
    m.naggs = 1;
    m.agg_op[0] = NUT_AGG_COUNT;
  }
  std::vector<int64_t> kw;
  std::vector<uint64_t> sw;
  nut_status st = run_groupby(c, m, hint, kw, sw, ng);
  if (st) return st;
  const int nkw = std::max(nwk, 1);
  // unpack the key tuples
  const size_t nk = std::max<size_t>(nkey, 1);
  keys.assign(ng * nk + 1, 0);
  for (uint64_t i = 0; i < ng; ++i)
    for (size_t j = 0; j < nkey; ++j) {
      const KeyField &k = fk[j];
      const uint64_t word = (uint64_t)kw[i * nkw + k.word];
      keys[i * nk + j] = k.bits >= 64 ? (int64_t)word
                                      : (int64_t)(((word >> k.shift) & ((1ull << k.bits) - 1)) + (uint64_t)k.mn);
    }
  words.assign(ng * na + 1, 0);
  for (size_t a = 0; a < na; ++a)
    if (gx.slot[a] >= 0)
      for (uint64_t i = 0; i < ng; ++i) words[i * na + a] = sw[i * m.naggs + gx.slot[a]];
  // countUnique: GROUP BY (key words, x) -> its groups on the device -> COUNT per key words
  for (size_t ci = 0; ci < cus.size() && ng; ++ci) {
    const int a = cus[ci];
    std::vector<KeyField> f1 = fk;
    f1.push_back(fx[ci]);
    int nw1 = 0;
    if (!layout_fields(f1, &nw1))
      return fail(NUT_ERR_UNSUPPORTED, "countUnique: the keys and its argument need more than 2 x 63 bits packed");
    nut_agg_spec q1 = s;
    q1.where = and_prog(s.where, gx.cu_mask[a], store);
    q1.nkeys = nw1;
    for (int w = 0; w < nw1; ++w) {
      st = word_prog(f1, w, -1, store, q1.key_prog[w]);
      if (st) return st;
    }
    q1.naggs = 1;
    memset(q1.agg_mask, 0, sizeof q1.agg_mask);
    memset(q1.agg_val, 0, sizeof q1.agg_val);
    q1.agg_op[0] = NUT_AGG_COUNT;
    // group hint: the main pass's groups times the argument's value range, capped at a
    // quarter of the rows and 2^26 (the result table is sized from it) — a high-cardinality
    // countUnique takes the partitioned path in one pass instead of regrowing an on-chip
    // table with a rescan per growth step
    const int xb = fx[ci].bits;
    const uint64_t xr = xb >= 40 ? (1ull << 40) : (1ull << xb);
    const uint64_t hcap = std::min<uint64_t>(s.n / 4, 1ull << 26);
    const uint64_t hint1 = std::max<uint64_t>(1, ng > hcap / xr ? hcap : std::min(hcap, ng * xr));
    nut_groups *g1 = nullptr;
    st = nut_groupby(c, &q1, hint1, &g1);
    if (st) return st;
    uint64_t n1 = 0;
    st = nut_groups_size(g1, &n1);
    DevBuf d1;
    if (!st && n1) {
      if (d1.alloc(c, (size_t)(nw1 + 1) * n1 * 8) != hipSuccess) st = fail(NUT_ERR_OOM, "hipMalloc (countUnique)");
      if (!st) st = nut_groups_to_device(g1, (uint64_t *)d1.p, n1);
    }
    nut_groups_free(g1);
    if (st) return st;
    std::vector<int64_t> k2;
    std::vector<uint64_t> w2;
    uint64_t n2 = 0;
    if (n1) {
      // the pass-1 groups' key words with x's bits cleared are the main pass's key words
      nut_agg_spec q2;
      memset(&q2, 0, sizeof q2);
      q2.n = n1;
      q2.prog_mode = 1;
      q2.nprog_cols = nw1;
      for (int w = 0; w < nw1; ++w) {
        q2.prog_col[w] = (const uint64_t *)d1.p + (size_t)w * n1;
        q2.prog_col_type[w] = NUT_T_I64;
      }
      const KeyField &x = f1.back();
      q2.nkeys = nwk;
      for (int w = 0; w < nwk; ++w) {
        store.nodes.emplace_back();
        std::vector<nut_prog_node> &v = store.nodes.back();
        v.push_back(nut_prog_node{NUT_P_COL, w, 0});
        if (x.word == w && x.bits < 64 && x.bits > 0) {
          v.push_back(nut_prog_node{NUT_P_I64, 0, (int64_t)~(((1ull << x.bits) - 1) << x.shift)});
          v.push_back(nut_prog_node{NUT_P_BITAND, 0, 0});
        }
        q2.key_prog[w] = nut_prog{(int32_t)v.size(), v.data()};
      }
      q2.naggs = 1;
      q2.agg_op[0] = NUT_AGG_COUNT;
      st = run_groupby(c, q2, ng, k2, w2, n2);
      if (st) return st;
    }
    // both group lists are sorted by key words: merge
    uint64_t j = 0;
    for (uint64_t i = 0; i < ng; ++i) {
      auto cmp = [&](uint64_t jj) {
        for (int w = 0; w < nwk; ++w) {
          const int64_t x0 = kw[i * nkw + w], y0 = k2[jj * nwk + w];
          if (x0 != y0) return x0 < y0 ? -1 : 1;
        }
        return 0;
      };
      while (j < n2 && nwk && cmp(j) > 0) ++j;
      words[i * na + a] = (j < n2 && (nwk == 0 || cmp(j) == 0)) ? w2[nwk ? j : 0] : 0;
    }
  }
  return NUT_OK;
}

// evaluation of an OUT_EXPR output for group i (nut_prog arithmetic semantics)
struct XVal {
  bool is_int;
  int64_t i;
  double f;
  double as_f() const { return is_int ? (double)i : f; }
};
XVal xpr_eval(const XNode &x, const std::vector<std::vector<uint64_t>> &cols, const std::vector<int> &types,
              uint64_t g, bool &div0) {
  if (x.k == X_CONST) return XVal{x.is_int, x.i, x.f};
  if (x.k == X_OUT) {
    const uint64_t w = cols[x.out][g];
    if (types[x.out] != NUT_T_F64) return XVal{true, (int64_t)w, 0.0};
    double f;
    memcpy(&f, &w, 8);
    return XVal{false, 0, f};
  }
  const XVal a = xpr_eval(x.kids[0], cols, types, g, div0);
  if (x.k == X_ABS) return a.is_int ? XVal{true, a.i < 0 ? (int64_t)(0 - (uint64_t)a.i) : a.i, 0.0} : XVal{false, 0, fabs(a.f)};
  if (x.k == X_TOF) return XVal{false, 0, a.as_f()};
  const XVal b = xpr_eval(x.kids[1], cols, types, g, div0);
  const bool ii = a.is_int && b.is_int;
  switch (x.k) {
    case X_ADD: return ii ? XVal{true, (int64_t)((uint64_t)a.i + (uint64_t)b.i), 0.0} : XVal{false, 0, a.as_f() + b.as_f()};
    case X_SUB: return ii ? XVal{true, (int64_t)((uint64_t)a.i - (uint64_t)b.i), 0.0} : XVal{false, 0, a.as_f() - b.as_f()};
    case X_MUL: return ii ? XVal{true, (int64_t)((uint64_t)a.i * (uint64_t)b.i), 0.0} : XVal{false, 0, a.as_f() * b.as_f()};
    case X_DIV: return XVal{false, 0, a.as_f() / b.as_f()};
    case X_MOD:
    case X_INTDIV:
      if (!ii) {
        if (x.k == X_INTDIV) {
          div0 = true;  // (reported as a plan error by the caller's type check)
          return XVal{false, 0, 0.0};
        }
        return XVal{false, 0, fmod(a.as_f(), b.as_f())};
      }
      if (b.i == 0) {
        div0 = true;
        return XVal{true, 0, 0.0};
      }
      if (b.i == -1) return XVal{true, x.k == X_MOD ? 0 : (int64_t)(0 - (uint64_t)a.i), 0.0};
      return XVal{true, x.k == X_MOD ? a.i % b.i : a.i / b.i, 0.0};
    default: return XVal{true, 0, 0.0};
  }
}
// static type of an OUT_EXPR (NUT_T_I64 / NUT_T_F64); -1: intDiv of a float64
int xpr_type(const XNode &x, const std::vector<int> &types) {
  if (x.k == X_CONST) return x.is_int ? NUT_T_I64 : NUT_T_F64;
  if (x.k == X_OUT) return types[x.out] == NUT_T_F64 ? NUT_T_F64 : NUT_T_I64;
  if (x.k == X_TOF || x.k == X_DIV) {
    for (const XNode &k : x.kids)
      if (xpr_type(k, types) < 0) return -1;
    return NUT_T_F64;
  }
  int t = NUT_T_I64;
  for (const XNode &k : x.kids) {
    const int tk = xpr_type(k, types);
    if (tk < 0) return -1;
    if (tk == NUT_T_F64) t = NUT_T_F64;
  }
  if (x.k == X_INTDIV && t == NUT_T_F64) return -1;
  return t;
}

// fkey[j]: GROUP BY key j is a float64 column bound to its key words (exec_groupby)
nut_status groupby_bound(nut_ctx *c, const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts,
                         uint64_t n, uint64_t hint, nut_result *r, const std::vector<char> &fkey) {
  nut_agg_spec s;
  ProgStore store;  // program nodes, alive until nut_groupby returns
  std::vector<int> agg_f64;
  GbExtra gx;
  nut_status bs = build_spec(p, bound, dicts, n, s, store, agg_f64, &gx);
  if (bs) return bs;
  uint64_t ng = 0;
  std::vector<int64_t> keys;
  std::vector<uint64_t> words;
  nut_status st = gx.active ? groupby_packed(c, p, s, gx, store, hint, keys, words, ng)
                            : run_groupby(c, s, hint, keys, words, ng);
  if (st) return st;
  const size_t nk = std::max<size_t>(p.keys.size(), 1), na = p.aggs.size();
  if (p.keys.empty() && ng == 0) {
    // a global aggregate over no rows is still one row: counts and sums 0, min/max 0,
    // avg NaN (ClickHouse's non-Nullable results)
    ng = 1;
    keys.assign(1, 0);
    words.assign(na + 1, 0);
  }
  // output columns in SELECT order (string keys stay codes until the end)
  r->host.resize(p.outs.size());
  std::vector<const Dict *> out_dict(p.outs.size(), nullptr);
  for (size_t j = 0; j < p.outs.size(); ++j) {
    const PlanOut &o = p.outs[j];
    std::vector<uint64_t> &col = r->host[j];
    col.resize(ng);
    int type = NUT_T_I64;
    if (o.kind == OUT_EXPR) {
      type = -1;  // below, once every other output is known
    } else if (o.kind == OUT_KEY) {
      const int dc = key_dict_col(p, (size_t)o.a);
      if (dicts && dc >= 0 && dicts[dc]) {
        type = NUT_T_STR;
        out_dict[j] = dicts[dc];
      }
      for (uint64_t i = 0; i < ng; ++i) col[i] = (uint64_t)keys[i * nk + o.a];
      if ((size_t)o.a < fkey.size() && fkey[o.a]) {  // key words -> the (canonical) float64 values
        type = NUT_T_F64;
        for (uint64_t &w : col) w ^= (uint64_t)((int64_t)w >> 63) >> 1;
      }
    } else if (o.kind == OUT_AGG) {
      type = agg_f64[o.a] ? NUT_T_F64 : NUT_T_I64;
      for (uint64_t i = 0; i < ng; ++i) col[i] = words[i * na + o.a];
    } else {
      type = NUT_T_F64;
      for (uint64_t i = 0; i < ng; ++i) {
        uint64_t sw = words[i * na + o.a];
        double sum;
        if (agg_f64[o.a])
          memcpy(&sum, &sw, 8);
        else
          sum = (double)(int64_t)sw;
        double avg = sum / (double)(int64_t)words[i * na + o.b];
        memcpy(&col[i], &avg, 8);
      }
    }
    r->names.push_back(o.name);
    r->types.push_back(type);
  }
  // arithmetic over the outputs (its operands are keys / aggregates / avg, never OUT_EXPR)
  for (size_t j = 0; j < p.outs.size(); ++j) {
    const PlanOut &o = p.outs[j];
    if (o.kind != OUT_EXPR) continue;
    const XNode &x = p.xprs[o.a];
    std::vector<const XNode *> todo{&x};
    while (!todo.empty()) {
      const XNode *y = todo.back();
      todo.pop_back();
      if (y->k == X_OUT && r->types[y->out] == NUT_T_STR)
        return fail(NUT_ERR_PLAN, "'" + o.text + "': arithmetic on the string key '" + p.outs[y->out].name + "'");
      for (const XNode &k : y->kids) todo.push_back(&k);
    }
    const int t = xpr_type(x, r->types);
    if (t < 0) return fail(NUT_ERR_PLAN, "'" + o.text + "': intDiv needs integer operands");
    bool div0 = false;
    for (uint64_t i = 0; i < ng; ++i) {
      const XVal v = xpr_eval(x, r->host, r->types, i, div0);
      if (t == NUT_T_I64) {
        r->host[j][i] = (uint64_t)v.i;
      } else {
        const double f = v.as_f();
        memcpy(&r->host[j][i], &f, 8);
      }
    }
    if (div0) return fail(NUT_ERR_INVALID_ARG, "'" + o.text + "': division by zero");
    r->types[j] = t;
  }
  // HAVING, then ORDER BY over outputs (groups arrive sorted by key tuple), then LIMIT
  if (p.has_having) {
    std::vector<const HNode *> todo{&p.having};
    while (!todo.empty()) {
      const HNode *h = todo.back();
      todo.pop_back();
      if (h->k == H_OUT && r->types[h->out] == NUT_T_STR)
        return fail(NUT_ERR_PLAN, "HAVING on the string key '" + p.outs[h->out].name + "' is not executed");
      for (const HNode &k : h->kids) todo.push_back(&k);
    }
  }
  auto str_of = [&](size_t j, uint64_t i) -> std::string {
    const std::string *t = out_dict[j]->decode((int64_t)r->host[j][i]);
    return t ? *t : std::string();
  };
  std::vector<uint64_t> idx;
  idx.reserve(ng);
  for (uint64_t i = 0; i < ng; ++i)
    if (!p.has_having || having_true(p.having, r->host, r->types, i)) idx.push_back(i);
  const uint64_t kept = idx.size();
  if (!p.order.empty()) {
    std::stable_sort(idx.begin(), idx.end(), [&](uint64_t x, uint64_t y) {
      for (const auto &ok : p.order) {
        const std::vector<uint64_t> &col = r->host[ok.first];
        int cmp;
        if (r->types[ok.first] == NUT_T_STR) {
          const int c2 = str_of(ok.first, x).compare(str_of(ok.first, y));
          cmp = c2 < 0 ? -1 : c2 > 0 ? 1 : 0;
        } else if (r->types[ok.first] == NUT_T_F64) {
          // the IEEE total order (-0.0 < +0.0, NaNs at the ends by sign), as the scans'
          // ORDER BY: a strict weak order even over NaN
          const uint64_t a = f64_to_ord(col[x]), b = f64_to_ord(col[y]);
          cmp = a < b ? -1 : a > b ? 1 : 0;
        } else {
          int64_t a = (int64_t)col[x], b = (int64_t)col[y];
          cmp = a < b ? -1 : a > b ? 1 : 0;
        }
        if (cmp) return ok.second ? cmp > 0 : cmp < 0;
      }
      return false;
    });
  }
  uint64_t off = p.has_limit ? std::min(p.offset, kept) : 0;
  uint64_t rows = kept - off;
  if (p.has_limit) rows = std::min(rows, p.limit);
  std::vector<std::vector<uint64_t>> vis;
  std::vector<std::string> names;
  std::vector<int> types;
  std::vector<std::vector<std::string>> strs;
  for (size_t j = 0; j < p.outs.size(); ++j) {
    if (p.outs[j].hidden) continue;
    std::vector<uint64_t> out(rows);
    for (uint64_t i = 0; i < rows; ++i) out[i] = r->host[j][idx[off + i]];
    strs.emplace_back();
    if (r->types[j] == NUT_T_STR)
      for (uint64_t i = 0; i < rows; ++i) strs.back().push_back(str_of(j, idx[off + i]));
    vis.push_back(std::move(out));
    names.push_back(r->names[j]);
    types.push_back(r->types[j]);
  }
  r->strs.swap(strs);
  r->host.swap(vis);
  r->names.swap(names);
  r->types.swap(types);
  r->nrows = rows;
  return NUT_OK;
}

// GROUP BY over float64 columns: each such key is grouped on a column of
// int64 words of its own — the IEEE total order with -0.0 = +0.0 and every NaN one value
// (f64_signed_order, canon; one 16 B/row pass per key) — so the group kernels, the packed
// key fields and the key-tuple order are the int64 ones, and the outputs decode the words
// back (+0.0 for the zeros, the quiet +NaN for the NaNs).  A WHERE or aggregate over the
// same column still reads its float64 values.
nut_status exec_groupby(nut_ctx *c, const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts,
                        uint64_t n, uint64_t hint, nut_result *r) {
  std::vector<char> fkey(p.keys.size(), 0);
  bool any = false;
  for (size_t j = 0; j < p.keys.size(); ++j)
    if (p.keys[j] >= 0 && bound[p.keys[j]]->type == NUT_T_F64 && !(dicts && dicts[p.keys[j]])) fkey[j] = 1, any = true;
  if (!any) return groupby_bound(c, p, bound, dicts, n, hint, r, fkey);
  nut_plan q = p;
  std::vector<const nut_column *> b(bound, bound + p.cols.size());
  std::vector<const Dict *> d(p.cols.size(), nullptr);
  if (dicts) d.assign(dicts, dicts + p.cols.size());
  std::deque<DevBuf> words;
  std::deque<nut_column> wcols;
  for (size_t j = 0; j < p.keys.size(); ++j) {
    if (!fkey[j]) continue;
    const nut_column *fc = bound[p.keys[j]];
    words.emplace_back();
    if (words.back().alloc(c, std::max<uint64_t>(n, 1) * 8) != hipSuccess) return fail(NUT_ERR_OOM, "hipMalloc (float64 keys)");
    nut_status st = f64_signed_order(c, (const uint64_t *)fc->data, (uint64_t *)words.back().p, p.never ? 0 : n, true);
    if (st) return st;
    wcols.push_back(nut_column{fc->name, words.back().p, NUT_T_I64});
    const int ci = (int)q.cols.size();
    q.cols.push_back("\x1f" "f64key:" + p.cols[p.keys[j]]);
    b.push_back(&wcols.back());
    d.push_back(nullptr);
    q.keys[j] = ci;
    if (j < q.key_progs.size() && q.key_progs[j].size() == 1 && q.key_progs[j][0].op == NUT_P_COL) q.key_progs[j][0].col = ci;
  }
  return groupby_bound(c, q, b.data(), d.data(), n, hint, r, fkey);
}

}  // namespace plan
}  // namespace nut
