/*
 * host_q1.c — a torch-free, Python-free host driving libnutexec.so through the C ABI
 * alone (include/nutexec.h), the way the Rust `extern "C"` block of INTEGRATION.md §3
 * would: hipMalloc'd columns, nut_ctx_create, the hot path, results to host, checked
 * against the C oracle (oracle/liboracle.so, test infrastructure).
 *
 *   1. config 4 (TPC-H Q1 shape): nut_gen_column x6 -> nut_q1 -> nut_groups_to_host
 *   2. the same query as SQL: nut_sql_plan -> nut_plan_execute -> nut_result_to_host
 *   3. config 2 filter and config 5 sort
 *   4. the library's own multi-GPU path: nut_dist_create (RCCL, ncclCommInitAll) over
 *      device 0 and nut_dist_create_virtual (3 ranks on device 0): group-by and sort
 *
 * Exit status 0 and one "host_q1 OK" line on success.  Built by tests/c/build.py with
 * gcc (no hipcc): plain C against the HIP runtime's C API.  Run by
 * tests/test_gpu_c_host.py, which also checks the process never mapped torch or Python.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nutexec.h"
#include "oracle.h"

#define N_ROWS 2000003ull
#define DATE_K 10471

static int failures = 0;

#define CHECK_NUT(call)                                                              \
  do {                                                                               \
    nut_status st_ = (call);                                                         \
    if (st_ != NUT_OK) {                                                             \
      fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #call, (int)st_,   \
              nut_last_error());                                                     \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)
#define CHECK_HIP(call)                                                              \
  do {                                                                               \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)
#define EXPECT(cond, ...)                  \
  do {                                     \
    if (!(cond)) {                         \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fputc('\n', stderr);                 \
      ++failures;                          \
    }                                      \
  } while (0)

static double as_f64(uint64_t w) {
  double d;
  memcpy(&d, &w, 8);
  return d;
}

/* 1 if this process mapped torch or a Python runtime (it must not: the point of the test) */
static int mapped_torch_or_python(void) {
  FILE *f = fopen("/proc/self/maps", "r");
  char line[4096];
  int found = 0;
  if (!f) return 0;
  while (fgets(line, sizeof line, f))
    if (strstr(line, "libtorch") || strstr(line, "libpython") || strstr(line, "libc10")) found = 1;
  fclose(f);
  return found;
}

static int rel_ok(uint64_t a, uint64_t b) {
  double x = as_f64(a), y = as_f64(b);
  return fabs(x - y) <= 1e-12 * fabs(y);
}

/* the Q1 columns of nutdb_amd/workloads.py Q1_COLS */
static const struct {
  int kind;
  uint64_t seed;
  int64_t a, b;
  double c;
} Q1[6] = {
    {NUT_GEN_RANGE_I64, 0x41, 8036, 2526, 1.0},       {NUT_GEN_RANGE_I64, 0x42, 0, 3, 1.0},
    {NUT_GEN_RANGE_I64, 0x43, 0, 2, 1.0},             {NUT_GEN_RANGE_F64, 0x44, 1, 50, 1.0},
    {NUT_GEN_RANGE_F64, 0x45, 90000, 10404901, 100.0}, {NUT_GEN_RANGE_F64, 0x46, 0, 11, 100.0},
};

int main(void) {
  int ndev = 0;
  CHECK_HIP(hipGetDeviceCount(&ndev));
  if (ndev < 1) {
    fprintf(stderr, "no GPU\n");
    return 2;
  }
  const uint64_t n = N_ROWS;
  nut_ctx *ctx = NULL;
  CHECK_NUT(nut_ctx_create(0, &ctx));

  /* ---------------------------------------------------------------- columns */
  void *dcol[6];
  void *hcol[6];
  for (int i = 0; i < 6; ++i) {
    CHECK_HIP(hipMalloc(&dcol[i], n * 8));
    hcol[i] = malloc(n * 8);
    CHECK_NUT(nut_gen_column(ctx, Q1[i].kind, Q1[i].seed, Q1[i].a, Q1[i].b, Q1[i].c, 0, n, dcol[i]));
    orc_gen_column(Q1[i].kind, Q1[i].seed, Q1[i].a, Q1[i].b, Q1[i].c, 0, n, hcol[i]);
  }

  /* ---------------------------------------------------------------- oracle Q1 */
  orc_agg_spec os;
  memset(&os, 0, sizeof(os));
  os.n = n;
  os.nkeys = 2;
  os.keys[0] = (const int64_t *)hcol[1];
  os.keys[1] = (const int64_t *)hcol[2];
  os.npred = 1;
  os.pred_col[0] = hcol[0];
  os.pred_type[0] = ORC_T_I64;
  os.pred_op[0] = ORC_LE;
  os.pred_i64[0] = DATE_K;
  os.nvals = 3;
  for (int i = 0; i < 3; ++i) os.val_col[i] = hcol[3 + i], os.val_type[i] = ORC_T_F64;
  os.naggs = 4;
  os.agg_op[0] = ORC_AGG_SUM, os.agg_expr[0] = ORC_EX_COL, os.agg_arg[0][0] = 0;
  os.agg_op[1] = ORC_AGG_SUM, os.agg_expr[1] = ORC_EX_COL, os.agg_arg[1][0] = 1;
  os.agg_op[2] = ORC_AGG_SUM, os.agg_expr[2] = ORC_EX_MUL_1M, os.agg_arg[2][0] = 1, os.agg_arg[2][1] = 2;
  os.agg_op[3] = ORC_AGG_COUNT;
  int64_t ok_[16];
  uint64_t ow[32];
  uint64_t og = orc_groupby(&os, 8, ok_, ow, 0);
  EXPECT(og == 6, "oracle Q1 groups %llu", (unsigned long long)og);

  /* ---------------------------------------------------------------- 1. nut_q1 */
  nut_groups *g = NULL;
  CHECK_NUT(nut_q1(ctx, dcol[0], dcol[1], dcol[2], dcol[3], dcol[4], dcol[5], n, DATE_K, &g));
  uint64_t ng = 0;
  CHECK_NUT(nut_groups_size(g, &ng));
  int64_t gk[16];
  uint64_t gw[32];
  EXPECT(ng == og, "nut_q1 groups %llu != %llu", (unsigned long long)ng, (unsigned long long)og);
  CHECK_NUT(nut_groups_to_host(g, gk, gw, 8));
  for (uint64_t i = 0; i < ng && i < og; ++i) {
    EXPECT(gk[2 * i] == ok_[2 * i] && gk[2 * i + 1] == ok_[2 * i + 1], "Q1 key %llu", (unsigned long long)i);
    for (int a = 0; a < 3; ++a) EXPECT(rel_ok(gw[4 * i + a], ow[4 * i + a]), "Q1 sum %d of group %llu", a, (unsigned long long)i);
    EXPECT(gw[4 * i + 3] == ow[4 * i + 3], "Q1 count of group %llu", (unsigned long long)i);
  }
  nut_groups_free(g);

  /* ---------------------------------------------------------------- 2. SQL */
  const char *sql =
      "select l_returnflag, l_linestatus, sum(l_quantity) as sum_qty, sum(l_extendedprice) as sum_base_price, "
      "sum(l_extendedprice * (1 - l_discount)) as sum_disc_price, count(*) as count_order from lineitem "
      "where l_shipdate <= toDate('1998-12-01') - interval 90 day "
      "group by l_returnflag, l_linestatus order by l_returnflag, l_linestatus";
  nut_plan *plan = NULL;
  CHECK_NUT(nut_sql_plan(sql, strlen(sql), &plan));
  const char *names[6] = {"l_shipdate", "l_returnflag", "l_linestatus", "l_quantity", "l_extendedprice", "l_discount"};
  nut_column cols[6];
  for (int i = 0; i < 6; ++i) {
    cols[i].name = names[i];
    cols[i].data = dcol[i];
    cols[i].type = i < 3 ? NUT_T_I64 : NUT_T_F64;
  }
  nut_result *res = NULL;
  CHECK_NUT(nut_plan_execute(ctx, plan, cols, 6, n, 8, &res));
  uint64_t rrows = 0;
  int rcols = 0;
  CHECK_NUT(nut_result_shape(res, &rrows, &rcols));
  EXPECT(rrows == og && rcols == 6, "SQL Q1 shape %llu x %d", (unsigned long long)rrows, rcols);
  if (rrows == og && rcols == 6) {
    int64_t rf[8], ls[8], cnt[8];
    uint64_t s[3][8];
    CHECK_NUT(nut_result_to_host(res, 0, rf, 8));
    CHECK_NUT(nut_result_to_host(res, 1, ls, 8));
    for (int a = 0; a < 3; ++a) CHECK_NUT(nut_result_to_host(res, 2 + a, s[a], 8));
    CHECK_NUT(nut_result_to_host(res, 5, cnt, 8));
    for (uint64_t i = 0; i < og; ++i) {
      EXPECT(rf[i] == ok_[2 * i] && ls[i] == ok_[2 * i + 1], "SQL key %llu", (unsigned long long)i);
      for (int a = 0; a < 3; ++a) EXPECT(rel_ok(s[a][i], ow[4 * i + a]), "SQL sum %d row %llu", a, (unsigned long long)i);
      EXPECT((uint64_t)cnt[i] == ow[4 * i + 3], "SQL count row %llu", (unsigned long long)i);
    }
  }
  nut_result_free(res);
  nut_plan_free(plan);

  /* ---------------------------------------------------------------- 3. filter + sort */
  int64_t *dk, *dout;
  CHECK_HIP(hipMalloc((void **)&dk, n * 8));
  CHECK_HIP(hipMalloc((void **)&dout, n * 8));
  int64_t *hk = (int64_t *)malloc(n * 8), *hout = (int64_t *)malloc(n * 8), *want = (int64_t *)malloc(n * 8);
  CHECK_NUT(nut_gen_column(ctx, NUT_GEN_U62, 0x2A, 0, 0, 1.0, 0, n, dk));
  orc_gen_column(ORC_GEN_U62, 0x2A, 0, 0, 1.0, 0, n, hk);
  uint64_t fn = 0;
  const int64_t k = (int64_t)1 << 61;
  CHECK_NUT(nut_filter_i64(ctx, dk, n, NUT_LT, k, dout, &fn));
  uint64_t wn = orc_filter_i64(hk, n, ORC_LT, k, want);
  EXPECT(fn == wn, "filter count %llu != %llu", (unsigned long long)fn, (unsigned long long)wn);
  CHECK_HIP(hipMemcpy(hout, dout, fn * 8, hipMemcpyDeviceToHost));
  EXPECT(fn == wn && memcmp(hout, want, fn * 8) == 0, "filter output differs");

  CHECK_NUT(nut_gen_column(ctx, NUT_GEN_FULL_I64, 0x50, 0, 0, 1.0, 0, n, dk));
  orc_gen_column(ORC_GEN_FULL_I64, 0x50, 0, 0, 1.0, 0, n, hk);
  CHECK_NUT(nut_sort_i64(ctx, dk, dout, n));
  CHECK_NUT(nut_ctx_sync(ctx));
  CHECK_HIP(hipMemcpy(hout, dout, n * 8, hipMemcpyDeviceToHost));
  orc_sort_i64(hk, want, n, 0);
  EXPECT(memcmp(hout, want, n * 8) == 0, "sort output differs");

  /* ---------------------------------------------------------------- 4. nut_dist */
  for (int mode = 0; mode < 2; ++mode) {
    nut_dist *d = NULL;
    int dev0 = 0;
    if (mode == 0)
      CHECK_NUT(nut_dist_create(1, &dev0, &d));
    else
      CHECK_NUT(nut_dist_create_virtual(3, 0, &d));
    int P = 0, L = 0, first = -1;
    CHECK_NUT(nut_dist_info(d, &P, &L, &first));
    EXPECT(P == (mode ? 3 : 1) && L == P && first == 0, "nut_dist_info %d %d %d", P, L, first);
    /* row shards of the Q1 columns: member l holds rows [l*n/P, (l+1)*n/P) */
    nut_agg_spec specs[3];
    for (int l = 0; l < P; ++l) {
      uint64_t r0 = n * l / P, r1 = n * (l + 1) / P;
      nut_agg_spec *s = &specs[l];
      memset(s, 0, sizeof(*s));
      s->n = r1 - r0;
      s->nkeys = 2;
      s->keys[0] = (const int64_t *)dcol[1] + r0;
      s->keys[1] = (const int64_t *)dcol[2] + r0;
      s->npred = 1;
      s->pred_col[0] = (const int64_t *)dcol[0] + r0;
      s->pred_type[0] = NUT_T_I64;
      s->pred_op[0] = NUT_LE;
      s->pred_i64[0] = DATE_K;
      s->nvals = 3;
      for (int i = 0; i < 3; ++i) s->val_col[i] = (const double *)dcol[3 + i] + r0, s->val_type[i] = NUT_T_F64;
      s->naggs = 4;
      s->agg_op[0] = NUT_AGG_SUM, s->agg_expr[0] = NUT_EX_COL, s->agg_arg[0][0] = 0;
      s->agg_op[1] = NUT_AGG_SUM, s->agg_expr[1] = NUT_EX_COL, s->agg_arg[1][0] = 1;
      s->agg_op[2] = NUT_AGG_SUM, s->agg_expr[2] = NUT_EX_MUL_1M, s->agg_arg[2][0] = 1, s->agg_arg[2][1] = 2;
      s->agg_op[3] = NUT_AGG_COUNT;
    }
    CHECK_NUT(nut_ctx_sync(ctx)); /* the columns were written on ctx's stream */
    nut_groups *out[3] = {NULL, NULL, NULL};
    CHECK_NUT(nut_dist_groupby(d, specs, 8, out));
    EXPECT(out[0] != NULL, "nut_dist_groupby: no result on rank 0");
    for (int l = 1; l < P; ++l) EXPECT(out[l] == NULL, "nut_dist_groupby: result on rank %d", l);
    if (out[0]) {
      CHECK_NUT(nut_groups_size(out[0], &ng));
      EXPECT(ng == og, "dist Q1 groups %llu", (unsigned long long)ng);
      CHECK_NUT(nut_groups_to_host(out[0], gk, gw, 8));
      for (uint64_t i = 0; i < ng && i < og; ++i) {
        EXPECT(gk[2 * i] == ok_[2 * i] && gk[2 * i + 1] == ok_[2 * i + 1], "dist Q1 key %llu", (unsigned long long)i);
        for (int a = 0; a < 3; ++a) EXPECT(rel_ok(gw[4 * i + a], ow[4 * i + a]), "dist Q1 sum %d", a);
        EXPECT(gw[4 * i + 3] == ow[4 * i + 3], "dist Q1 count");
      }
      nut_groups_free(out[0]);
    }
    /* sample sort of the sort column's shards */
    const int64_t *ins[3], *outs[3];
    uint64_t ns[3], on[3];
    for (int l = 0; l < P; ++l) {
      uint64_t r0 = n * l / P, r1 = n * (l + 1) / P;
      ins[l] = dk + r0;
      ns[l] = r1 - r0;
    }
    CHECK_NUT(nut_dist_sort_i64(d, ins, ns, outs, on));
    uint64_t pos = 0;
    for (int l = 0; l < P; ++l) {
      EXPECT(pos + on[l] <= n, "dist sort: too many keys");
      if (pos + on[l] > n) break;
      CHECK_NUT(nut_ctx_memcpy(nut_dist_ctx(d, l), hout + pos, outs[l], on[l] * 8));
      pos += on[l];
    }
    EXPECT(pos == n && memcmp(hout, want, n * 8) == 0, "dist sort: concatenation is not the sorted input");
    nut_dist_destroy(d);
  }

  for (int i = 0; i < 6; ++i) {
    (void)hipFree(dcol[i]);
    free(hcol[i]);
  }
  (void)hipFree(dk);
  (void)hipFree(dout);
  free(hk);
  free(hout);
  free(want);
  nut_ctx_destroy(ctx);
  EXPECT(!mapped_torch_or_python(), "torch or Python is mapped into the C host");
  if (failures) {
    fprintf(stderr, "host_q1: %d failures\n", failures);
    return 1;
  }
  printf("host_q1 OK: Q1 %llu groups (nut_q1, SQL, nut_dist RCCL + 3 virtual ranks), filter %llu rows, sort %llu keys\n",
         (unsigned long long)og, (unsigned long long)fn, (unsigned long long)n);
  return 0;
}
