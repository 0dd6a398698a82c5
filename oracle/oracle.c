/*
 * oracle.c — CPU restatement of the nutexec hot path.  TEST INFRASTRUCTURE ONLY
 * (see oracle.h for who may load it and how it is pinned).
 *
 * Written as the plainest correct loops: one pass per operator, OpenMP over row
 * chunks, per-thread hash tables merged at the end, Neumaier-compensated f64 sums.
 * Nothing here shares code with nutdb_amd/csrc (the HIP product path).
 *
 * Anchors in the reference (the AST the executor consumes; /root/reference):
 *   WHERE  -> src/parser/ast/query.rs:68-72 (WhereClause{condition: Expr})
 *   GROUP  -> src/parser/ast/query.rs:74-78 (GroupByClause{keys})
 *   SELECT -> src/parser/ast/query.rs:25 (columns) with FnCall sum/count/min/max
 *             (src/parser/ast/expr.rs:32-36; names are FnName::Others, item.rs:164-179)
 *   ORDER  -> src/parser/ast/query.rs:86-90 (OrderByClause)
 * The operators themselves have no reference implementation.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

int orc_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* counter-based splitmix64 — identical bits in C, numpy, HIP. */
uint64_t orc_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t orc_gen_u64(uint64_t seed, uint64_t row) {
  return orc_mix64(seed + (row + 1) * 0x9E3779B97F4A7C15ull);
}

void orc_gen_column(int kind, uint64_t seed, int64_t a, int64_t b, double c,
                    uint64_t row0, uint64_t n, void *out) {
  int64_t *oi = (int64_t *)out;
  double *od = (double *)out;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    uint64_t u = orc_gen_u64(seed, row0 + (uint64_t)i);
    switch (kind) {
      case ORC_GEN_U62: oi[i] = (int64_t)(u >> 2); break;
      case ORC_GEN_FULL_I64: oi[i] = (int64_t)u; break;
      case ORC_GEN_POOL_KEY: oi[i] = (int64_t)orc_mix64((u % (uint64_t)a) ^ ORC_POOL_SALT); break;
      case ORC_GEN_DYADIC: od[i] = (double)(u >> 44) / 64.0; break;
      case ORC_GEN_UNIT_F64: od[i] = (double)(u >> 11) * 0x1p-53; break;
      case ORC_GEN_RANGE_I64: oi[i] = a + (int64_t)(u % (uint64_t)b); break;
      case ORC_GEN_RANGE_F64: od[i] = (double)(a + (int64_t)(u % (uint64_t)b)) / c; break;
      case ORC_GEN_SKEW_KEY: oi[i] = (int64_t)orc_mix64(ORC_SKEW_INDEX(u, a) ^ ORC_POOL_SALT); break;
      default: oi[i] = 0;
    }
  }
}

/* ------------------------------------------------------------------ filter */
static int cmp_i64(int64_t v, int op, int64_t k) {
  switch (op) {
    case ORC_LT: return v < k;
    case ORC_LE: return v <= k;
    case ORC_GT: return v > k;
    case ORC_GE: return v >= k;
    case ORC_EQ: return v == k;
    default: return v != k;
  }
}
static int cmp_f64(double v, int op, double k) {
  switch (op) {
    case ORC_LT: return v < k;
    case ORC_LE: return v <= k;
    case ORC_GT: return v > k;
    case ORC_GE: return v >= k;
    case ORC_EQ: return v == k;
    default: return v != k;
  }
}

uint64_t orc_filter_i64(const int64_t *col, uint64_t n, int op, int64_t k, int64_t *out) {
  int nt = orc_max_threads();
  uint64_t *cnt = (uint64_t *)calloc((size_t)nt + 1, sizeof(uint64_t));
  uint64_t chunk = (n + (uint64_t)nt - 1) / (uint64_t)nt;
#pragma omp parallel num_threads(nt)
  {
#ifdef _OPENMP
    int t = omp_get_thread_num();
#else
    int t = 0;
#endif
    uint64_t lo = (uint64_t)t * chunk, hi = lo + chunk > n ? n : lo + chunk;
    uint64_t c = 0;
    for (uint64_t i = lo; i < hi; ++i) c += (uint64_t)cmp_i64(col[i], op, k);
    cnt[t + 1] = c;
#pragma omp barrier
#pragma omp single
    for (int j = 0; j < nt; ++j) cnt[j + 1] += cnt[j];
    uint64_t w = cnt[t];
    if (out)
      for (uint64_t i = lo; i < hi; ++i)
        if (cmp_i64(col[i], op, k)) out[w++] = col[i];
  }
  uint64_t total = cnt[nt];
  free(cnt);
  return total;
}

/* ----------------------------------------------------------------- group-by */
/* total order on f64 bit patterns (-0 < +0; NaN above +inf) — the documented
 * MIN/MAX semantics of nutexec */
static uint64_t f64_ord(double d) {
  uint64_t b;
  memcpy(&b, &d, 8);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

typedef struct {
  int64_t k[2];
  uint64_t w[8];   /* aggregate words */
  double comp[8];  /* Neumaier compensation for f64 sums */
  double sumf[8];  /* running f64 sum (kept as double to compensate) */
} grp_t;

typedef struct {
  uint64_t cap, n;
  int64_t *slot;   /* index into g, -1 empty */
  grp_t *g;
  uint64_t gcap;
} table_t;

static uint64_t hash_keys(const int64_t *k, int nk) {
  uint64_t h = orc_mix64((uint64_t)k[0] ^ 0x243F6A8885A308D3ull);
  if (nk == 2) h = orc_mix64(h ^ (uint64_t)k[1]);
  return h;
}

static void tbl_init(table_t *t, uint64_t cap) {
  t->cap = cap;
  t->n = 0;
  t->slot = (int64_t *)malloc(cap * sizeof(int64_t));
  memset(t->slot, 0xff, cap * sizeof(int64_t));
  t->gcap = cap / 2 + 1;
  t->g = (grp_t *)malloc(t->gcap * sizeof(grp_t));
}
static void tbl_free(table_t *t) {
  free(t->slot);
  free(t->g);
}

static void grp_init(grp_t *g, const orc_agg_spec *s, const int64_t *k) {
  g->k[0] = k[0];
  g->k[1] = s->nkeys == 2 ? k[1] : 0;
  for (int a = 0; a < s->naggs; ++a) {
    g->comp[a] = 0.0;
    g->sumf[a] = 0.0;
    int isf = s->agg_op[a] != ORC_AGG_COUNT &&
              !(s->agg_expr[a] == ORC_EX_COL && s->val_type[s->agg_arg[a][0]] == ORC_T_I64);
    switch (s->agg_op[a]) {
      case ORC_AGG_SUM: g->w[a] = 0; break;
      case ORC_AGG_COUNT: g->w[a] = 0; break;
      case ORC_AGG_MIN: g->w[a] = isf ? ~0ull : (uint64_t)INT64_MAX; break;
      default: g->w[a] = isf ? 0ull : (uint64_t)INT64_MIN; break;
    }
  }
}

static grp_t *tbl_find(table_t *t, const orc_agg_spec *s, const int64_t *k);

static void tbl_grow(table_t *t, const orc_agg_spec *s) {
  uint64_t ncap = t->cap * 2;
  int64_t *ns = (int64_t *)malloc(ncap * sizeof(int64_t));
  memset(ns, 0xff, ncap * sizeof(int64_t));
  for (uint64_t i = 0; i < t->n; ++i) {
    uint64_t h = hash_keys(t->g[i].k, s->nkeys) & (ncap - 1);
    while (ns[h] >= 0) h = (h + 1) & (ncap - 1);
    ns[h] = (int64_t)i;
  }
  free(t->slot);
  t->slot = ns;
  t->cap = ncap;
  t->gcap = ncap / 2 + 1;
  t->g = (grp_t *)realloc(t->g, t->gcap * sizeof(grp_t));
}

static grp_t *tbl_find(table_t *t, const orc_agg_spec *s, const int64_t *k) {
  uint64_t h = hash_keys(k, s->nkeys) & (t->cap - 1);
  for (;;) {
    int64_t idx = t->slot[h];
    if (idx < 0) break;
    grp_t *g = &t->g[idx];
    if (g->k[0] == k[0] && (s->nkeys == 1 || g->k[1] == k[1])) return g;
    h = (h + 1) & (t->cap - 1);
  }
  if (t->n + 1 > t->cap / 2) {
    tbl_grow(t, s);
    return tbl_find(t, s, k);
  }
  t->slot[h] = (int64_t)t->n;
  grp_t *g = &t->g[t->n++];
  grp_init(g, s, k);
  return g;
}

static void neumaier_add(double *sum, double *comp, double x) {
  double t = *sum + x;
  if (fabs(*sum) >= fabs(x))
    *comp += (*sum - t) + x;
  else
    *comp += (x - t) + *sum;
  *sum = t;
}

static double eval_f64(const orc_agg_spec *s, int a, uint64_t i) {
  const double *c0 = (const double *)s->val_col[s->agg_arg[a][0]];
  double x = c0[i];
  switch (s->agg_expr[a]) {
    case ORC_EX_COL: return x;
    case ORC_EX_MUL: return x * ((const double *)s->val_col[s->agg_arg[a][1]])[i];
    case ORC_EX_ADD: return x + ((const double *)s->val_col[s->agg_arg[a][1]])[i];
    case ORC_EX_SUB: return x - ((const double *)s->val_col[s->agg_arg[a][1]])[i];
    case ORC_EX_MUL_1M: {
      double b = ((const double *)s->val_col[s->agg_arg[a][1]])[i];
      volatile double t = 1.0 - b; /* no contraction: exactly two roundings */
      return x * t;
    }
    default: {
      double b = ((const double *)s->val_col[s->agg_arg[a][1]])[i];
      double c = ((const double *)s->val_col[s->agg_arg[a][2]])[i];
      volatile double t1 = 1.0 - b;
      volatile double t2 = x * t1;
      volatile double t3 = 1.0 + c;
      return t2 * t3;
    }
  }
}

static int row_passes(const orc_agg_spec *s, uint64_t i) {
  if (s->row_mask && !s->row_mask[i]) return 0;
  for (int p = 0; p < s->npred; ++p) {
    if (s->pred_type[p] == ORC_T_I64) {
      if (!cmp_i64(((const int64_t *)s->pred_col[p])[i], s->pred_op[p], s->pred_i64[p])) return 0;
    } else {
      if (!cmp_f64(((const double *)s->pred_col[p])[i], s->pred_op[p], s->pred_f64[p])) return 0;
    }
  }
  return 1;
}

static int agg_is_i64(const orc_agg_spec *s, int a) {
  return s->agg_op[a] != ORC_AGG_COUNT && s->agg_expr[a] == ORC_EX_COL &&
         s->val_type[s->agg_arg[a][0]] == ORC_T_I64;
}

static void grp_update(grp_t *g, const orc_agg_spec *s, uint64_t i) {
  for (int a = 0; a < s->naggs; ++a) {
    int op = s->agg_op[a];
    if (s->agg_mask[a] && !s->agg_mask[a][i]) continue;
    if (op == ORC_AGG_COUNT) {
      g->w[a] += 1;
      continue;
    }
    if (agg_is_i64(s, a)) {
      int64_t v = ((const int64_t *)s->val_col[s->agg_arg[a][0]])[i];
      if (op == ORC_AGG_SUM) g->w[a] = g->w[a] + (uint64_t)v; /* wraps */
      else if (op == ORC_AGG_MIN) { if (v < (int64_t)g->w[a]) g->w[a] = (uint64_t)v; }
      else { if (v > (int64_t)g->w[a]) g->w[a] = (uint64_t)v; }
      continue;
    }
    double v = eval_f64(s, a, i);
    if (op == ORC_AGG_SUM) neumaier_add(&g->sumf[a], &g->comp[a], v);
    else if (op == ORC_AGG_MIN) { uint64_t o = f64_ord(v); if (o < g->w[a]) g->w[a] = o; }
    else { uint64_t o = f64_ord(v); if (o > g->w[a]) g->w[a] = o; }
  }
}

static void grp_merge(grp_t *dst, const grp_t *src, const orc_agg_spec *s) {
  for (int a = 0; a < s->naggs; ++a) {
    int op = s->agg_op[a];
    if (op == ORC_AGG_COUNT) { dst->w[a] += src->w[a]; continue; }
    if (agg_is_i64(s, a)) {
      if (op == ORC_AGG_SUM) dst->w[a] += src->w[a];
      else if (op == ORC_AGG_MIN) { if ((int64_t)src->w[a] < (int64_t)dst->w[a]) dst->w[a] = src->w[a]; }
      else { if ((int64_t)src->w[a] > (int64_t)dst->w[a]) dst->w[a] = src->w[a]; }
      continue;
    }
    if (op == ORC_AGG_SUM) {
      neumaier_add(&dst->sumf[a], &dst->comp[a], src->sumf[a]);
      dst->comp[a] += src->comp[a];
    } else if (op == ORC_AGG_MIN) { if (src->w[a] < dst->w[a]) dst->w[a] = src->w[a]; }
    else { if (src->w[a] > dst->w[a]) dst->w[a] = src->w[a]; }
  }
}

static int cmp_grp(const void *pa, const void *pb, void *nkp) {
  const grp_t *a = (const grp_t *)pa, *b = (const grp_t *)pb;
  int nk = *(int *)nkp;
  if (a->k[0] != b->k[0]) return a->k[0] < b->k[0] ? -1 : 1;
  if (nk == 2 && a->k[1] != b->k[1]) return a->k[1] < b->k[1] ? -1 : 1;
  return 0;
}

static int g_sort_nk;
static int cmp_grp_q(const void *a, const void *b) { return cmp_grp(a, b, &g_sort_nk); }

/* the group's result words (f64 sums folded with their compensation, MIN / MAX of f64
 * back from the ordered encoding) */
static void grp_out(const grp_t *g, const orc_agg_spec *s, int64_t *ok, uint64_t *ow) {
  ok[0] = g->k[0];
  if (s->nkeys == 2) ok[1] = g->k[1];
  for (int a = 0; a < s->naggs; ++a) {
    uint64_t w = g->w[a];
    int op = s->agg_op[a];
    if (op != ORC_AGG_COUNT && !agg_is_i64(s, a)) {
      double d;
      if (op == ORC_AGG_SUM) {
        d = g->sumf[a] + g->comp[a];
      } else {
        uint64_t b = (w >> 63) ? (w & 0x7FFFFFFFFFFFFFFFull) : ~w;
        memcpy(&d, &b, 8);
      }
      memcpy(&w, &d, 8);
    }
    ow[a] = w;
  }
}

/* key tuple order (signed, lexicographic) */
static int tuple_lt(const int64_t *a, const int64_t *b, int nk) {
  if (a[0] != b[0]) return a[0] < b[0];
  return nk == 2 && a[1] < b[1];
}
static int cmp_tuple(const void *pa, const void *pb) {
  const int64_t *a = (const int64_t *)pa, *b = (const int64_t *)pb;
  if (a[0] != b[0]) return a[0] < b[0] ? -1 : 1;
  if (g_sort_nk == 2 && a[1] != b[1]) return a[1] < b[1] ? -1 : 1;
  return 0;
}

/* Large group counts: the same result as the per-thread tables below, computed without
 * their serial merge.  Rows are range-partitioned by key tuple (P - 1 splitters from a
 * sorted row sample); each partition then runs on one thread with tables that fit its
 * cache: per partition, the rows of thread chunk t (the chunks orc_groupby uses) fold in
 * row order into a fresh table, which merges into the partition's result in chunk order —
 * exactly the per-group order of the per-thread tables and their merge into table 0 (a
 * group merged into a fresh group is that group, bit for bit), so the two paths agree
 * bitwise.  Partitions are key ranges, so each one's groups sorted and laid out in
 * partition order are the global order.  Returns UINT64_MAX - 1 when the sample shows few
 * groups (the per-thread tables are faster there). */
/* distinct key tuples of s's rows (all rows, WHERE ignored): k-minimum-values — each
 * thread keeps the KMV_K smallest distinct tuple hashes of its chunk (sorted; a hash above
 * the current k-th is rejected in O(1), which is almost every row), the union's k-th
 * smallest h_k gives (k - 1) / (h_k / 2^64); fewer than k distinct hashes: their count */
#define KMV_K 1024
static int cmp_u64(const void *pa, const void *pb) {
  const uint64_t a = *(const uint64_t *)pa, b = *(const uint64_t *)pb;
  return a < b ? -1 : a > b;
}
static double kmv_distinct(const orc_agg_spec *s, int nt) {
  const uint64_t n = s->n, chunk = (n + (uint64_t)nt - 1) / (uint64_t)nt;
  uint64_t *mins = (uint64_t *)malloc((size_t)nt * KMV_K * sizeof(uint64_t));
  int *cnt = (int *)calloc((size_t)nt, sizeof(int));
#pragma omp parallel num_threads(nt)
  {
#ifdef _OPENMP
    int t = omp_get_thread_num();
#else
    int t = 0;
#endif
    const uint64_t lo = (uint64_t)t * chunk, hi = lo + chunk > n ? n : lo + chunk;
    uint64_t *a = mins + (size_t)t * KMV_K;
    int c = 0;
    for (uint64_t i = lo; i < hi; ++i) {
      const int64_t k[2] = {s->keys[0][i], s->nkeys == 2 ? s->keys[1][i] : 0};
      const uint64_t h = orc_mix64(hash_keys(k, s->nkeys) ^ 0x9E3779B97F4A7C15ull);
      if (c == KMV_K && h >= a[KMV_K - 1]) continue;
      int lo2 = 0, hi2 = c;  /* first position with a[pos] >= h */
      while (lo2 < hi2) {
        const int mid = (lo2 + hi2) >> 1;
        if (a[mid] < h) lo2 = mid + 1;
        else hi2 = mid;
      }
      if (lo2 < c && a[lo2] == h) continue;  /* seen */
      const int keep = c < KMV_K ? c : KMV_K - 1;
      memmove(a + lo2 + 1, a + lo2, (size_t)(keep - lo2) * sizeof(uint64_t));
      a[lo2] = h;
      if (c < KMV_K) ++c;
    }
    cnt[t] = c;
  }
  /* union: the k smallest distinct over the threads' lists */
  uint64_t *u = (uint64_t *)malloc((size_t)nt * KMV_K * sizeof(uint64_t));
  size_t nu = 0;
  for (int t = 0; t < nt; ++t)
    for (int j = 0; j < cnt[t]; ++j) u[nu++] = mins[(size_t)t * KMV_K + j];
  qsort(u, nu, sizeof(uint64_t), cmp_u64);
  size_t d = 0;
  for (size_t j = 0; j < nu; ++j)
    if (!d || u[j] != u[d - 1]) u[d++] = u[j];
  double est = (double)d;
  if (d >= KMV_K) est = (double)(KMV_K - 1) / ((double)u[KMV_K - 1] / 18446744073709551616.0);
  free(u);
  free(mins);
  free(cnt);
  return est;
}

#define ORC_HEAVY_MAX 64
static uint64_t groupby_ranges(const orc_agg_spec *s, uint64_t cap, int64_t *out_keys, uint64_t *out_aggs, int nt) {
  const uint64_t n = s->n, chunk = (n + (uint64_t)nt - 1) / (uint64_t)nt;
  const int nk = s->nkeys;
  if (nk < 1 || n < ((uint64_t)1 << 22)) return UINT64_MAX - 1;
  /* a strided sample of the tuples: the few-groups gate, the heavy tuples and the splitters */
  const uint64_t m = 65536;
  int64_t *smp = (int64_t *)malloc(m * 2 * sizeof(int64_t));
  for (uint64_t j = 0; j < m; ++j) {
    const uint64_t i = (uint64_t)(((unsigned __int128)j * n) / m);
    smp[2 * j] = s->keys[0][i];
    smp[2 * j + 1] = nk == 2 ? s->keys[1][i] : 0;
  }
  g_sort_nk = nk;
  qsort(smp, m, 2 * sizeof(int64_t), cmp_tuple);
  /* few groups, seen in the sample: every sampled tuple occurs at least twice (no more than
   * 1/64 of them once) and there are few of them — the per-thread tables, without the sketch
   * (whose binary-search inserts never stop below k distinct hashes: G = 1000 ran 4x slower
   * through it) */
  {
    uint64_t d = 0, f1 = 0;
    for (uint64_t j = 0; j < m;) {
      uint64_t e = j + 1;
      while (e < m && cmp_tuple(&smp[2 * j], &smp[2 * e]) == 0) ++e;
      ++d;
      f1 += e - j == 1;
      j = e;
    }
    if (f1 * 64 <= d && d * 16 <= m) {
      free(smp);
      return UINT64_MAX - 1;
    }
  }
  /* ---- distinct groups: a k-minimum-values sketch over every key tuple (one hashing pass;
   * ~3 % error at k = 1024).  The strided sample's Chao1 estimate it replaces is a lower
   * bound that skew breaks: Zipf-like keys over 4.6 M groups estimated ~1.3e5 and went to
   * the per-thread tables, whose serial merge of millions of groups ran 3x slower than the
   * ranges. */
  const double gest = kmv_distinct(s, nt);
  if (gest < 262144) {  /* (per-thread tables of <= ~2^18 groups stay cache-resident and merge fast:
                          G = 1e5 ran 3.1e8 rows/s there vs 1.3e8 through the ranges) */
    free(smp);
    return UINT64_MAX - 1;
  }
  /* ---- heavy tuples: a sample run of >= 1/nt of the sample is more rows than one thread's
   * share, and a key range holding it would leave its partition on one thread (skewed keys
   * ran 5x slower than uniform ones).  Each thread folds its chunk's rows of such a tuple in
   * row order into a group of its own (pass 1) — exactly that chunk's group in the
   * partition's per-chunk table — and the chunks' groups merge in chunk order into a fresh
   * group, which joins its key range's partition as one more fresh group: the same words,
   * bit for bit, as without the split.  The splitters come from the other sample rows. */
  int nh = 0;
  int64_t hk[2 * ORC_HEAVY_MAX];
  uint64_t m2 = 0;
  for (uint64_t j = 0; j < m;) {
    uint64_t e = j + 1;
    while (e < m && cmp_tuple(&smp[2 * j], &smp[2 * e]) == 0) ++e;
    if (nt > 1 && (e - j) * (uint64_t)nt >= m && nh < ORC_HEAVY_MAX) {
      hk[2 * nh] = smp[2 * j];
      hk[2 * nh + 1] = smp[2 * j + 1];
      ++nh;
    } else {
      for (uint64_t r = j; r < e; ++r, ++m2) {
        smp[2 * m2] = smp[2 * r];
        smp[2 * m2 + 1] = smp[2 * r + 1];
      }
    }
    j = e;
  }
  int P = 2;
  while (P < 4096 && (double)P * 4096 < gest) P *= 2;
  while (P > 1 && (uint64_t)P * 16 > m2) P /= 2;  /* (few light sample rows: few partitions) */
  int64_t *spl = (int64_t *)malloc((size_t)P * 2 * sizeof(int64_t));  /* P - 1 splitters */
  for (int p = 1; p < P; ++p) {
    const uint64_t j = (uint64_t)p * m2 / (uint64_t)P;
    spl[2 * (p - 1)] = smp[2 * j];
    spl[2 * (p - 1) + 1] = smp[2 * j + 1];
  }
  free(smp);
  /* the heavy tuples' lookup (open addressing, 4x their number) and each one's partition */
  int hslot[4 * ORC_HEAVY_MAX];
  int hpart[ORC_HEAVY_MAX];
  for (int q = 0; q < 4 * ORC_HEAVY_MAX; ++q) hslot[q] = -1;
  for (int j = 0; j < nh; ++j) {
    uint64_t q = hash_keys(&hk[2 * j], nk) & (4 * ORC_HEAVY_MAX - 1);
    while (hslot[q] >= 0) q = (q + 1) & (4 * ORC_HEAVY_MAX - 1);
    hslot[q] = j;
    int a = 0, b = P - 1;
    while (a < b) {
      const int mid = (a + b) >> 1;
      if (tuple_lt(&hk[2 * j], &spl[2 * mid], nk)) b = mid;
      else a = mid + 1;
    }
    hpart[j] = a;
  }
  grp_t *hg = (grp_t *)malloc(((size_t)nt * (size_t)nh + 1) * sizeof(grp_t));  /* [t][j] chunk groups */
  unsigned char *hhit = (unsigned char *)calloc((size_t)nt * (size_t)nh + 1, 1);
  for (int t = 0; t < nt; ++t)
    for (int j = 0; j < nh; ++j) grp_init(&hg[(size_t)t * nh + j], s, &hk[2 * j]);
  /* ---- pass 1: each passing row's partition (#splitters <= its tuple), counts per (t, p) */
  uint16_t *pid = (uint16_t *)malloc(n * sizeof(uint16_t));
  uint64_t *cnt = (uint64_t *)calloc((size_t)nt * (size_t)P + 1, sizeof(uint64_t));
#pragma omp parallel num_threads(nt)
  {
#ifdef _OPENMP
    int t = omp_get_thread_num();
#else
    int t = 0;
#endif
    const uint64_t lo = (uint64_t)t * chunk, hi = lo + chunk > n ? n : lo + chunk;
    uint64_t *c = cnt + (size_t)t * (size_t)P;
    for (uint64_t i = lo; i < hi; ++i) {
      if (!row_passes(s, i)) {
        pid[i] = 0xFFFF;
        continue;
      }
      const int64_t k[2] = {s->keys[0][i], nk == 2 ? s->keys[1][i] : 0};
      if (nh) {
        uint64_t q = hash_keys(k, nk) & (4 * ORC_HEAVY_MAX - 1);
        int j = -1;
        for (; hslot[q] >= 0; q = (q + 1) & (4 * ORC_HEAVY_MAX - 1))
          if (hk[2 * hslot[q]] == k[0] && (nk == 1 || hk[2 * hslot[q] + 1] == k[1])) {
            j = hslot[q];
            break;
          }
        if (j >= 0) {  /* a heavy tuple: this chunk's group of it, in row order */
          grp_update(&hg[(size_t)t * nh + j], s, i);
          hhit[(size_t)t * nh + j] = 1;
          pid[i] = 0xFFFF;
          continue;
        }
      }
      int a = 0, b = P - 1; /* first splitter > k, in [0, P - 1] */
      while (a < b) {
        const int mid = (a + b) >> 1;
        if (tuple_lt(k, &spl[2 * mid], nk)) b = mid;
        else a = mid + 1;
      }
      pid[i] = (uint16_t)a;
      ++c[a];
    }
  }
  free(spl);
  /* partition-major layout: partition p's rows, thread chunk by thread chunk, row order */
  uint64_t *base = (uint64_t *)malloc(((size_t)P * (size_t)nt + 1) * sizeof(uint64_t));
  uint64_t run = 0;
  for (int p = 0; p < P; ++p)
    for (int t = 0; t < nt; ++t) {
      base[(size_t)p * nt + t] = run;
      run += cnt[(size_t)t * P + p];
    }
  base[(size_t)P * nt] = run;
  uint64_t *idx = (uint64_t *)malloc((run ? run : 1) * sizeof(uint64_t));
#pragma omp parallel num_threads(nt)
  {
#ifdef _OPENMP
    int t = omp_get_thread_num();
#else
    int t = 0;
#endif
    const uint64_t lo = (uint64_t)t * chunk, hi = lo + chunk > n ? n : lo + chunk;
    uint64_t *w = cnt + (size_t)t * (size_t)P; /* reused as this thread's write cursors */
    for (int p = 0; p < P; ++p) w[p] = base[(size_t)p * nt + t];
    for (uint64_t i = lo; i < hi; ++i)
      if (pid[i] != 0xFFFF) idx[w[pid[i]]++] = i;
  }
  free(pid);
  /* the heavy tuples' groups: chunk groups merged in chunk order into a fresh group */
  grp_t *hsum = (grp_t *)malloc(((size_t)nh + 1) * sizeof(grp_t));
  unsigned char *hany = (unsigned char *)calloc((size_t)nh + 1, 1);
  for (int j = 0; j < nh; ++j) {
    grp_init(&hsum[j], s, &hk[2 * j]);
    for (int t = 0; t < nt; ++t)
      if (hhit[(size_t)t * nh + j]) {
        grp_merge(&hsum[j], &hg[(size_t)t * nh + j], s);
        hany[j] = 1;
      }
  }
  free(hg);
  free(hhit);
  /* ---- pass 2: one partition per thread at a time */
  grp_t **pg = (grp_t **)calloc((size_t)P, sizeof(grp_t *));
  uint64_t *pn = (uint64_t *)calloc((size_t)P + 1, sizeof(uint64_t));
  g_sort_nk = nk;
#pragma omp parallel num_threads(nt)
  {
    table_t A, B;
    tbl_init(&A, 1024);
    tbl_init(&B, 1024);
#pragma omp for schedule(dynamic, 1)
    for (int p = 0; p < P; ++p) {
      A.n = 0;
      memset(A.slot, 0xff, A.cap * sizeof(int64_t));
      for (int t = 0; t < nt; ++t) {
        const uint64_t r0 = base[(size_t)p * nt + t], r1 = base[(size_t)p * nt + t + 1];
        if (r0 == r1) continue;
        B.n = 0;
        memset(B.slot, 0xff, B.cap * sizeof(int64_t));
        for (uint64_t r = r0; r < r1; ++r) {
          const uint64_t i = idx[r];
          const int64_t k[2] = {s->keys[0][i], nk == 2 ? s->keys[1][i] : 0};
          grp_update(tbl_find(&B, s, k), s, i);
        }
        for (uint64_t j = 0; j < B.n; ++j) grp_merge(tbl_find(&A, s, B.g[j].k), &B.g[j], s);
      }
      for (int j = 0; j < nh; ++j)  /* the heavy tuples of this key range (no other row of theirs is here) */
        if (hany[j] && hpart[j] == p) grp_merge(tbl_find(&A, s, hsum[j].k), &hsum[j], s);
      qsort(A.g, A.n, sizeof(grp_t), cmp_grp_q);
      pg[p] = (grp_t *)malloc((A.n ? A.n : 1) * sizeof(grp_t));
      memcpy(pg[p], A.g, A.n * sizeof(grp_t));
      pn[p] = A.n;
    }
    tbl_free(&A);
    tbl_free(&B);
  }
  free(idx);
  free(base);
  free(cnt);
  free(hsum);
  free(hany);
  uint64_t ng = 0;
  for (int p = 0; p < P; ++p) ng += pn[p];
  if (ng <= cap) {
    uint64_t *off = (uint64_t *)malloc((size_t)P * sizeof(uint64_t));
    for (int p = 0; p < P; ++p) off[p] = p ? off[p - 1] + pn[p - 1] : 0;
#pragma omp parallel for schedule(dynamic, 4) num_threads(nt)
    for (int p = 0; p < P; ++p)
      for (uint64_t j = 0; j < pn[p]; ++j)
        grp_out(&pg[p][j], s, out_keys + (off[p] + j) * (uint64_t)nk, out_aggs + (off[p] + j) * (uint64_t)s->naggs);
    free(off);
  }
  for (int p = 0; p < P; ++p) free(pg[p]);
  free(pg);
  free(pn);
  return ng <= cap ? ng : UINT64_MAX;
}

uint64_t orc_groupby(const orc_agg_spec *s, uint64_t cap, int64_t *out_keys,
                     uint64_t *out_aggs, int nthreads) {
  int nt = nthreads > 0 ? nthreads : orc_max_threads();
  const uint64_t r = groupby_ranges(s, cap, out_keys, out_aggs, nt);
  return r != UINT64_MAX - 1 ? r : orc_groupby_tables(s, cap, out_keys, out_aggs, nt);
}

/* per-thread tables over row chunks, merged into thread 0's in thread order, then sorted */
uint64_t orc_groupby_tables(const orc_agg_spec *s, uint64_t cap, int64_t *out_keys,
                            uint64_t *out_aggs, int nthreads) {
  int nt = nthreads > 0 ? nthreads : orc_max_threads();
  table_t *tl = (table_t *)calloc((size_t)nt, sizeof(table_t));
  uint64_t n = s->n, chunk = (n + (uint64_t)nt - 1) / (uint64_t)nt;
#pragma omp parallel num_threads(nt)
  {
#ifdef _OPENMP
    int t = omp_get_thread_num();
#else
    int t = 0;
#endif
    table_t *T = &tl[t];
    tbl_init(T, 1024);
    uint64_t lo = (uint64_t)t * chunk, hi = lo + chunk > n ? n : lo + chunk;
    int64_t k[2] = {0, 0};
    for (uint64_t i = lo; i < hi; ++i) {
      if (!row_passes(s, i)) continue;
      k[0] = s->keys[0][i];
      if (s->nkeys == 2) k[1] = s->keys[1][i];
      grp_update(tbl_find(T, s, k), s, i);
    }
  }
  table_t *G = &tl[0];
  for (int t = 1; t < nt; ++t) {
    for (uint64_t i = 0; i < tl[t].n; ++i) {
      grp_t *src = &tl[t].g[i];
      /* find-or-create in G, then merge */
      uint64_t before = G->n;
      grp_t *dst = tbl_find(G, s, src->k);
      (void)before;
      grp_merge(dst, src, s);
    }
    tbl_free(&tl[t]);
  }
  uint64_t ng = G->n;
  if (ng > cap) {
    tbl_free(G);
    free(tl);
    return UINT64_MAX;
  }
  g_sort_nk = s->nkeys;
  qsort(G->g, ng, sizeof(grp_t), cmp_grp_q);
  for (uint64_t i = 0; i < ng; ++i)
    grp_out(&G->g[i], s, out_keys + i * (uint64_t)s->nkeys, out_aggs + i * (uint64_t)s->naggs);
  tbl_free(G);
  free(tl);
  return ng;
}

/* --------------------------------------------------------------------- sort */
void orc_sort_i64(const int64_t *in, int64_t *out, uint64_t n, int nthreads) {
  int nt = nthreads > 0 ? nthreads : orc_max_threads();
  uint64_t *a = (uint64_t *)malloc(n * sizeof(uint64_t));
  uint64_t *b = (uint64_t *)malloc(n * sizeof(uint64_t));
#pragma omp parallel for num_threads(nt)
  for (int64_t i = 0; i < (int64_t)n; ++i) a[i] = (uint64_t)in[i] ^ 0x8000000000000000ull;
  uint64_t *hist = (uint64_t *)malloc((size_t)nt * 256 * sizeof(uint64_t));
  uint64_t chunk = (n + (uint64_t)nt - 1) / (uint64_t)nt;
  for (int pass = 0; pass < 8; ++pass) {
    int sh = pass * 8;
#pragma omp parallel num_threads(nt)
    {
#ifdef _OPENMP
      int t = omp_get_thread_num();
#else
      int t = 0;
#endif
      uint64_t *h = hist + (size_t)t * 256;
      memset(h, 0, 256 * sizeof(uint64_t));
      uint64_t lo = (uint64_t)t * chunk, hi = lo + chunk > n ? n : lo + chunk;
      for (uint64_t i = lo; i < hi; ++i) h[(a[i] >> sh) & 255]++;
#pragma omp barrier
#pragma omp single
      {
        uint64_t run = 0;
        for (int d = 0; d < 256; ++d)
          for (int tt = 0; tt < nt; ++tt) {
            uint64_t c = hist[(size_t)tt * 256 + d];
            hist[(size_t)tt * 256 + d] = run;
            run += c;
          }
      }
      for (uint64_t i = lo; i < hi; ++i) b[h[(a[i] >> sh) & 255]++] = a[i];
    }
    uint64_t *tmp = a; a = b; b = tmp;
  }
#pragma omp parallel for num_threads(nt)
  for (int64_t i = 0; i < (int64_t)n; ++i) out[i] = (int64_t)(a[i] ^ 0x8000000000000000ull);
  free(hist);
  free(a);
  free(b);
}

/* ------------------------------------------------------- expression programs */
enum { EO_COL = 0, EO_I64 = 1, EO_ADD = 3, EO_SUB = 4, EO_MUL = 5, EO_LT = 9, EO_LE, EO_GT, EO_GE, EO_EQ, EO_NE,
       EO_AND = 15, EO_OR, EO_XOR, EO_NOT, EO_BAND, EO_BOR, EO_BXOR, EO_BNOT, EO_IF = 25 };
#define EO_BLOCK 2048
#define EO_STACK 32

int orc_eval_int(const int32_t *op, const int32_t *arg, const int64_t *v, int nnodes, const int64_t *const *cols,
                 int ncols, uint64_t n, int64_t *out) {
  int depth = 0, maxd = 0;
  for (int j = 0; j < nnodes; ++j) {  /* validate: the subset, the stack, the columns */
    const int o = op[j];
    int k;
    if (o == EO_COL || o == EO_I64) k = 0;
    else if (o == EO_NOT || o == EO_BNOT) k = 1;
    else if (o == EO_IF) k = 3;
    else if (o == EO_ADD || o == EO_SUB || o == EO_MUL || (o >= EO_LT && o <= EO_NE) || o == EO_AND || o == EO_OR ||
             o == EO_XOR || o == EO_BAND || o == EO_BOR || o == EO_BXOR) k = 2;
    else return -1;
    if (o == EO_COL && (arg[j] < 0 || arg[j] >= ncols)) return -1;
    if (depth < k) return -1;
    depth = depth - k + 1;
    if (depth > maxd) maxd = depth;
  }
  if (depth != 1 || maxd > EO_STACK) return -1;
  const uint64_t nb = (n + EO_BLOCK - 1) / EO_BLOCK;
#pragma omp parallel
  {
    int64_t *st = (int64_t *)malloc((size_t)EO_STACK * EO_BLOCK * sizeof(int64_t));
#pragma omp for schedule(static)
    for (int64_t b = 0; b < (int64_t)nb; ++b) {
      const uint64_t lo = (uint64_t)b * EO_BLOCK, m = n - lo < EO_BLOCK ? n - lo : EO_BLOCK;
      int sp = 0;
      for (int j = 0; j < nnodes; ++j) {
        const int o = op[j];
        int64_t *r;
        if (o == EO_COL || o == EO_I64) {
          r = st + (size_t)sp++ * EO_BLOCK;
          if (o == EO_COL) memcpy(r, cols[arg[j]] + lo, m * sizeof(int64_t));
          else for (uint64_t i = 0; i < m; ++i) r[i] = v[j];
          continue;
        }
        if (o == EO_NOT || o == EO_BNOT) {
          r = st + (size_t)(sp - 1) * EO_BLOCK;
          if (o == EO_NOT) for (uint64_t i = 0; i < m; ++i) r[i] = r[i] == 0;
          else for (uint64_t i = 0; i < m; ++i) r[i] = ~r[i];
          continue;
        }
        if (o == EO_IF) {
          sp -= 2;
          int64_t *c = st + (size_t)(sp - 1) * EO_BLOCK, *x = c + EO_BLOCK, *y = x + EO_BLOCK;
          for (uint64_t i = 0; i < m; ++i) c[i] = c[i] ? x[i] : y[i];
          continue;
        }
        --sp;
        int64_t *a = st + (size_t)(sp - 1) * EO_BLOCK, *y = a + EO_BLOCK;
        switch (o) {
          case EO_ADD: for (uint64_t i = 0; i < m; ++i) a[i] = (int64_t)((uint64_t)a[i] + (uint64_t)y[i]); break;
          case EO_SUB: for (uint64_t i = 0; i < m; ++i) a[i] = (int64_t)((uint64_t)a[i] - (uint64_t)y[i]); break;
          case EO_MUL: for (uint64_t i = 0; i < m; ++i) a[i] = (int64_t)((uint64_t)a[i] * (uint64_t)y[i]); break;
          case EO_LT: for (uint64_t i = 0; i < m; ++i) a[i] = a[i] < y[i]; break;
          case EO_LE: for (uint64_t i = 0; i < m; ++i) a[i] = a[i] <= y[i]; break;
          case EO_GT: for (uint64_t i = 0; i < m; ++i) a[i] = a[i] > y[i]; break;
          case EO_GE: for (uint64_t i = 0; i < m; ++i) a[i] = a[i] >= y[i]; break;
          case EO_EQ: for (uint64_t i = 0; i < m; ++i) a[i] = a[i] == y[i]; break;
          case EO_NE: for (uint64_t i = 0; i < m; ++i) a[i] = a[i] != y[i]; break;
          case EO_AND: for (uint64_t i = 0; i < m; ++i) a[i] = (a[i] != 0) & (y[i] != 0); break;
          case EO_OR: for (uint64_t i = 0; i < m; ++i) a[i] = (a[i] != 0) | (y[i] != 0); break;
          case EO_XOR: for (uint64_t i = 0; i < m; ++i) a[i] = (a[i] != 0) != (y[i] != 0); break;
          case EO_BAND: for (uint64_t i = 0; i < m; ++i) a[i] &= y[i]; break;
          case EO_BOR: for (uint64_t i = 0; i < m; ++i) a[i] |= y[i]; break;
          default: for (uint64_t i = 0; i < m; ++i) a[i] ^= y[i]; break;
        }
      }
      memcpy(out + lo, st, m * sizeof(int64_t));
    }
    free(st);
  }
  return 0;
}

uint64_t orc_multiset_hash_i64(const int64_t *v, uint64_t n) {
  uint64_t h = 0;
#pragma omp parallel for reduction(+ : h)
  for (int64_t i = 0; i < (int64_t)n; ++i) h += orc_mix64((uint64_t)v[i] ^ 0xA0761D6478BD642Full);
  return h;
}

/* ------------------------------------------------- indexed pool-key group-by */
/* The synthetic config-3 key of row r is mix64((u_k(r) % G) ^ POOL_SALT): mix64 is a
 * bijection, so the pool index g = u_k(r) % G names the group.  The rows are accumulated
 * into dense per-thread [G] arrays indexed by g — no hashing, and for dyadic values
 * ((u_v >> 44) / 64) the sums are kept as integer 1/64 units, exact in any order (1e9 rows
 * x 2^20 units < 2^53).  Keys are regenerated from g and the groups ordered by key. */
typedef struct {
  int64_t key;
  uint64_t g;
} orc_kg;

static int kg_cmp(const void *a, const void *b) {
  const int64_t x = ((const orc_kg *)a)->key, y = ((const orc_kg *)b)->key;
  return x < y ? -1 : x > y;
}

uint64_t orc_groupby_pool_dyadic(uint64_t key_seed, uint64_t groups, uint64_t val_seed, uint64_t row0, uint64_t n,
                                 int64_t *out_keys, uint64_t *out_words, int nthreads) {
  return orc_groupby_pool_dyadic_kind(ORC_GEN_POOL_KEY, key_seed, groups, val_seed, row0, n, out_keys, out_words,
                                      nthreads);
}

uint64_t orc_groupby_pool_dyadic_kind(int kind, uint64_t key_seed, uint64_t groups, uint64_t val_seed, uint64_t row0,
                                      uint64_t n, int64_t *out_keys, uint64_t *out_words, int nthreads) {
  if (groups == 0) return 0;
  int nt = nthreads > 0 ? nthreads : orc_max_threads();
  const uint64_t G = groups;
  uint64_t *sum = (uint64_t *)calloc((size_t)nt * G, 8);
  uint64_t *cnt = (uint64_t *)calloc((size_t)nt * G, 8);
  uint32_t *mn = (uint32_t *)malloc((size_t)nt * G * 4);
  uint32_t *mx = (uint32_t *)calloc((size_t)nt * G, 4);
  if (!sum || !cnt || !mn || !mx) {
    free(sum); free(cnt); free(mn); free(mx);
    return UINT64_MAX;
  }
  memset(mn, 0xFF, (size_t)nt * G * 4);
  const uint64_t chunk = (n + (uint64_t)nt - 1) / (uint64_t)nt;
#pragma omp parallel num_threads(nt)
  {
#ifdef _OPENMP
    const int t = omp_get_thread_num();
#else
    const int t = 0;
#endif
    uint64_t *s = sum + (size_t)t * G, *c = cnt + (size_t)t * G;
    uint32_t *lo = mn + (size_t)t * G, *hi = mx + (size_t)t * G;
    const uint64_t a = (uint64_t)t * chunk, b = a + chunk > n ? n : a + chunk;
    for (uint64_t i = a; i < b; ++i) {
      const uint64_t u = orc_gen_u64(key_seed, row0 + i);
      const uint64_t g = kind == ORC_GEN_SKEW_KEY ? ORC_SKEW_INDEX(u, G) : u % G;
      const uint32_t v = (uint32_t)(orc_gen_u64(val_seed, row0 + i) >> 44);
      s[g] += v;
      c[g] += 1;
      if (v < lo[g]) lo[g] = v;
      if (v > hi[g]) hi[g] = v;
    }
  }
  /* merge into thread 0's arrays */
#pragma omp parallel for num_threads(nt) schedule(static)
  for (int64_t g = 0; g < (int64_t)G; ++g)
    for (int t = 1; t < nt; ++t) {
      const size_t j = (size_t)t * G + (size_t)g;
      sum[g] += sum[j];
      cnt[g] += cnt[j];
      if (mn[j] < mn[g]) mn[g] = mn[j];
      if (mx[j] > mx[g]) mx[g] = mx[j];
    }
  orc_kg *kg = (orc_kg *)malloc((size_t)G * sizeof(orc_kg));
  uint64_t m = 0;
  for (uint64_t g = 0; g < G; ++g)
    if (cnt[g]) {
      kg[m].key = (int64_t)orc_mix64(g ^ ORC_POOL_SALT);
      kg[m].g = g;
      ++m;
    }
  qsort(kg, (size_t)m, sizeof(orc_kg), kg_cmp);
#pragma omp parallel for num_threads(nt) schedule(static)
  for (int64_t i = 0; i < (int64_t)m; ++i) {
    const uint64_t g = kg[i].g;
    const double fs = (double)sum[g] / 64.0, fmn = (double)mn[g] / 64.0, fmx = (double)mx[g] / 64.0;
    out_keys[i] = kg[i].key;
    memcpy(&out_words[4 * i + 0], &fs, 8);
    out_words[4 * i + 1] = cnt[g];
    memcpy(&out_words[4 * i + 2], &fmn, 8);
    memcpy(&out_words[4 * i + 3], &fmx, 8);
  }
  free(kg); free(sum); free(cnt); free(mn); free(mx);
  return m;
}

/* Hash equi-join (include/nutexec.h nut_join_i64 semantics; join types 0 INNER, 1 LEFT,
 * 2 SEMI, 3 ANTI): a CSR bucket table over the build keys (OpenMP count / scan / fill),
 * then an OpenMP probe in two passes per thread chunk (count pairs, write them), so the
 * pairs come out in probe-row order.  Within a probe row the build rows are in the
 * table's fill order (unspecified).  Writes at most `cap` pairs; returns the pair count
 * (call again with a larger cap when it exceeds cap).  Pinned by the numpy join oracle
 * (oracle.py join_i64) in tests/test_join_cpu.py; the CPU baseline of bench.py join. */
static uint64_t join_bucket(int64_t k, int log2b) {
  return log2b ? orc_mix64((uint64_t)k ^ 0x3C6EF372FE94F82Aull) >> (64 - log2b) : 0;
}

uint64_t orc_join_i64(const int64_t *build, uint64_t nb, const int64_t *probe, uint64_t np, int type,
                      int64_t *out_p, int64_t *out_b, uint64_t cap) {
  int log2b = 0;
  while ((1ull << log2b) < 2 * nb) ++log2b;
  const uint64_t nbk = 1ull << log2b;
  uint64_t *off = calloc(nbk + 1, sizeof(uint64_t));
  int64_t *bkeys = malloc((nb ? nb : 1) * sizeof(int64_t)), *brow = malloc((nb ? nb : 1) * sizeof(int64_t));
#pragma omp parallel for
  for (int64_t i = 0; i < (int64_t)nb; ++i) {
    const uint64_t b = join_bucket(build[i], log2b);
#pragma omp atomic
    off[b + 1]++;
  }
  for (uint64_t b = 0; b < nbk; ++b) off[b + 1] += off[b];
  uint64_t *cur = malloc(nbk * sizeof(uint64_t));
  memcpy(cur, off, nbk * sizeof(uint64_t));
#pragma omp parallel for
  for (int64_t i = 0; i < (int64_t)nb; ++i) {
    const uint64_t b = join_bucket(build[i], log2b);
    uint64_t pos;
#pragma omp atomic capture
    pos = cur[b]++;
    bkeys[pos] = build[i];
    brow[pos] = i;
  }
  free(cur);
  const int nt = omp_get_max_threads();
  uint64_t *tcnt = calloc((size_t)nt + 1, sizeof(uint64_t));
  uint64_t total = 0;
#pragma omp parallel num_threads(nt)
  {
    const int t = omp_get_thread_num(), T = omp_get_num_threads();
    const uint64_t chunk = (np + T - 1) / T, lo = (uint64_t)t * chunk < np ? (uint64_t)t * chunk : np;
    const uint64_t hi = lo + chunk < np ? lo + chunk : np;
    uint64_t c = 0;
    for (uint64_t r = lo; r < hi; ++r) {
      const uint64_t b = join_bucket(probe[r], log2b);
      uint64_t m = 0;
      for (uint64_t j = off[b]; j < off[b + 1]; ++j) m += bkeys[j] == probe[r];
      c += type == 0 ? m : type == 1 ? (m ? m : 1) : type == 2 ? (m ? 1 : 0) : (m ? 0 : 1);
    }
    tcnt[t + 1] = c;
#pragma omp barrier
#pragma omp single
    {
      for (int i = 0; i < T; ++i) tcnt[i + 1] += tcnt[i];
      total = tcnt[T];
    }
    if (total <= cap) {
      uint64_t pos = tcnt[t];
      for (uint64_t r = lo; r < hi; ++r) {
        const int64_t k = probe[r];
        const uint64_t b = join_bucket(k, log2b);
        uint64_t m = 0;
        for (uint64_t j = off[b]; j < off[b + 1]; ++j)
          if (bkeys[j] == k) {
            if (type <= 1) {
              out_p[pos] = (int64_t)r;
              out_b[pos++] = brow[j];
            }
            ++m;
          }
        if ((type == 1 && !m) || (type == 2 && m) || (type == 3 && !m)) {
          out_p[pos] = (int64_t)r;
          out_b[pos++] = -1;
        }
      }
    }
  }
  free(tcnt);
  free(off);
  free(bkeys);
  free(brow);
  return total;
}
