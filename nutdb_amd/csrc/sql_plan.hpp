// sql_plan.hpp — internal to the SQL plan translation units (sql_lower.cpp, sql_exec_scan.cpp,
// sql_exec_groupby.cpp, sql_exec_join.cpp, sql_plan.cpp): the plan's data structures and
// the functions one unit calls in another.  Not part of the C ABI (include/nutexec.h).
#pragma once
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <tuple>

#include "common.hpp"
#include "sort.hpp"
#include "sql_ast.hpp"
#include "sql_lexer.hpp"
#include "table.hpp"

struct nut_stmt {
  std::string sql;   // the tree's views point into this copy
  nut::sql::Statement st;
};

namespace nut {
namespace plan {
using namespace nut::sql;

typedef __int128 i128;
// ------------------------------------------------------------------ constants
constexpr i128 kHuge = (i128)1 << 100;  // saturation bound: anything beyond is "out of every range"
struct CVal {
  bool is_int = true;
  i128 v = 0;        // integer value (saturated to +/-kHuge)
  Decimal dec;       // float value
  bool is_str = false;  // string constant (binds to a dictionary code at execution)
  std::string s;
  int param = -1;       // >= 0: the value of scalar subquery nut_plan.subs[param], known at execution
};
struct Lowering {
  std::string err;
  bool fail(const std::string &m) {
    if (err.empty()) err = m;
    return false;
  }
};
struct PlanPred {
  int col, op;
  CVal c;
  std::vector<CVal> set;  // NUT_IN / NUT_NOT_IN
};
// expression-program node before binding (compiled mode; nut_prog_op)
struct PNode {
  int op = NUT_P_I64;
  int col = -1;  // NUT_P_COL: plan column
  CVal c;        // NUT_P_I64 / NUT_P_F64 constant
  int arg = 0;   // NUT_P_DATEPART: nut_date_part; P_SUBSTR: the 1-based byte offset
};
using PProg = std::vector<PNode>;

struct PlanAgg {
  int op, expr;
  int arg[3];
  PProg val, mask;        // compiled mode: argument program and row mask (empty = every row)
  std::vector<int> refs;  // compiled mode: columns the argument reads (COUNT(x) included)
  bool distinct = false;  // countUnique(val): distinct values per group (op COUNT; two passes)
};
// Arithmetic over a group's outputs (SELECT sum(a) / count(), 100 * sum(x) / sum(y), ...),
// evaluated on the host per result group with nut_prog semantics: int + - * wrap, an f64
// operand makes the op f64, / is always f64, % and intDiv truncate (a zero divisor fails).
enum XKind { X_CONST, X_OUT, X_ADD, X_SUB, X_MUL, X_DIV, X_MOD, X_INTDIV, X_ABS, X_TOF };
struct XNode {
  int k = X_CONST;
  int out = -1;  // X_OUT: output index (a key, an aggregate or avg)
  bool is_int = true;
  int64_t i = 0;
  double f = 0;
  std::vector<XNode> kids;
};
enum OutKind { OUT_KEY, OUT_AGG, OUT_AVG, OUT_EXPR };
struct PlanOut {
  int kind, a, b;
  std::string name, text;
  bool hidden = false;  // computed for HAVING only, not part of the result
};

// HAVING, evaluated on the host over the (small) group result
enum HKind { H_CONST, H_OUT, H_CMP, H_AND, H_OR, H_NOT, H_BOOL };
struct HNode {
  int k = H_BOOL;
  int op = 0;        // H_CMP: nut_cmp
  int out = -1;      // H_OUT: output index
  bool is_int = false, b = true;
  int64_t i = 0;
  double f = 0;
  int param = -1;    // H_CONST: >= 0, the value of scalar subquery nut_plan.subs[param]
  std::vector<HNode> kids;
};

extern const char *kCmpText[];
}  // namespace plan
}  // namespace nut

using namespace nut;
using namespace nut::sql;
using namespace nut::plan;


// FULL OUTER JOIN (plans only): executed as a LEFT join plus the JOIN source's unmatched
// rows (an ANTI join with the roles swapped); the kernels know types 0..3
constexpr int PJ_FULL = 4;
// RIGHT OUTER as a step of a chain (the JOIN source preserved, every earlier table
// NULL-extended); a single RIGHT JOIN is a LEFT join with jright
constexpr int PJ_RIGHT = 5;
// GROUP BY keys of one plan (packed into the kernels' two key words)
constexpr int kMaxGroupKeys = 8;

struct nut_plan {
  int kind = NUT_PLAN_FILTER;
  bool compiled = false;          // expression mode: WHERE / aggregate arguments are programs
  PProg where;                    // compiled mode WHERE (empty = every row)
  std::string table;
  std::vector<std::string> cols;  // names the plan binds
  bool never = false;             // WHERE folded to false
  std::vector<PlanPred> preds;
  int proj = -1;                  // FILTER/SORT column (the first projected one)
  std::vector<int> projs;         // every projected column (expression-mode scans: several; computed: -1)
  std::vector<PProg> proj_val, proj_mask;  // per projection: its program and NULL mask (plain columns: empty)
  std::vector<int> isnull_cols;   // columns under an IS [NOT] NULL (folded to a constant)
  bool star = false;              // SELECT *: every bound column, expanded at execution (expand_star)
  bool desc = false;              // SORT direction
  // SORT: the ORDER BY keys as (plan column, desc), most significant first.  One key equal
  // to the only projected column: a keys-only sort; otherwise row ids are sorted by the
  // keys (stable pair sorts, last key first) and every projected column gathered.
  std::vector<std::pair<int, bool>> sort_keys;
  std::vector<int> keys, vals;    // GROUPBY key / value columns (indices into cols; a computed key: -1)
  // GROUPBY keys (compiled mode): each key's program (a plain key: COL) and expression text
  // (to match SELECT items); up to kMaxGroupKeys, packed into two words at execution
  std::vector<PProg> key_progs;
  std::vector<std::string> key_text;
  std::vector<XNode> xprs;        // OUT_EXPR outputs' expressions
  std::vector<PlanAgg> aggs;
  std::vector<PlanOut> outs;
  std::vector<std::pair<int, bool>> order;  // GROUPBY: (output, desc)
  bool has_having = false;
  HNode having;
  bool has_limit = false;
  uint64_t limit = 0, offset = 0;
  // JOIN (one JoinClause with ON a = b), executed by nut_plan_execute2: a hash join
  // (nut_join_i64) then gathers into the joined table the rest of the plan runs on
  int join = -1;           // nut_join_type, or PJ_FULL; -1: no JOIN
  // several INNER JoinClauses (nut_plan_executen): table k+1 joins on jn[k].key
  struct JoinStep {
    std::string table, alias;
    int key[2] = {-1, -1};      // plan columns of the ON equality (EXISTS: found at execution)
    int type = NUT_JOIN_INNER;  // NUT_JOIN_INNER / LEFT / SEMI / ANTI, PJ_RIGHT, PJ_FULL
    // A correlated EXISTS / NOT EXISTS or [NOT] IN (subquery): a SEMI /
    // ANTI step over the subquery's table.  scope >= 1 names the subquery: its unqualified
    // names are plan columns of that scope (scoped_name) and bind to its table first.
    // cond = its WHERE conjuncts, split at execution (when each column's table is known)
    // into pushed-down filters of the subquery's table, the correlation equality (the
    // key, EXISTS) and at most one other comparison with the outer query (the residual).
    int scope = 0;
    PProg cond;
  };
  std::vector<JoinStep> jn;
  bool jright = false;     // RIGHT OUTER / SEMI / ANTI: the JOIN source is the preserved side
  std::string jtable, talias, jalias;  // JOIN source; FROM / JOIN aliases (qualifiers)
  int jkey[2] = {-1, -1};  // plan columns of the ON equality
  std::deque<std::string> qnames;  // storage of qualified column names (column_ref)
  // JOIN ... USING (u): the plain name u, and the qualified column it stands for
  std::vector<std::pair<std::string, std::string>> using_cols;
  // uncorrelated scalar subqueries `(SELECT agg(..) FROM t WHERE ..)` compared in WHERE /
  // HAVING or used as a value: global-aggregate plans over the same table, executed first;
  // their one value replaces every constant whose param names them (resolve_subqueries)
  std::vector<std::shared_ptr<nut_plan>> subs;
  int scope = 0;  // lowering state: the EXISTS / IN subquery whose names are being lowered
  // FROM (SELECT .. GROUP BY ..) d, or a CTE of that shape: the derived
  // table is materialized — `inner` executes over the caller's columns first and this plan
  // runs over its result columns (bound by output name)
  std::shared_ptr<nut_plan> inner;
  // UNION ALL: the branches, each its own single-table plan, run in order
  // and their results concatenated; this plan mirrors branch 0's kind, and `cols` lists
  // every branch's columns once (what nut_plan_execute binds; nut_plan_executen gives
  // branch k the k-th table)
  std::vector<std::shared_ptr<nut_plan>> uni;
};

struct nut_result {
  int kind = NUT_PLAN_FILTER;
  int device = 0;
  uint64_t nrows = 0;
  std::vector<std::string> names;
  std::vector<int> types;
  void *dev = nullptr;  // FILTER/SORT: owned device buffer
  uint64_t dev_off = 0;
  uint64_t dev_stride = 0;  // FILTER with several columns: column j at dev + j * dev_stride
  std::vector<std::vector<uint64_t>> host;  // GROUPBY: output columns (int64 / f64 bits)
  std::vector<std::vector<std::string>> strs;  // NUT_T_STR columns, decoded (others empty)
  // SQL NULLs (FILTER/SORT): column j's 1-byte flags at valid + valid_of[j] * dev_stride +
  // dev_off (valid_of[j] < 0 or empty: no NULLs)
  uint8_t *valid = nullptr;
  std::vector<int> valid_of;
};


namespace nut {
namespace plan {

// internal program leaves (never reach nut_prog): `col [I]LIKE 'pattern'` over a
// dictionary column, lowered at execution to COL + LOOKUP in a per-code match table;
// `substring(col, arg, c.v)` over one (c.v = kHuge: to the end), lowered at execution to
// COL + MAP from the column's codes to its substrings' codes in the same dictionary
constexpr int P_LIKE = 1000, P_ILIKE = 1001, P_SUBSTR = 1002;
// a node that reads its plan column (col)
inline bool reads_col(int op) { return op == NUT_P_COL || op == P_LIKE || op == P_ILIKE || op == P_SUBSTR; }
// ------------------------------------------------------------------ predicate resolution
enum Verdict { V_PRED, V_TRUE, V_FALSE };
// a query-lifetime device buffer: stream-ordered (hipMallocAsync on the context's stream,
// whose pool keeps freed memory — nut_ctx_create), so the per-query selections, join
// indices and gathered columns cost no hipMalloc / hipFree round trip
struct DevBuf {
  void *p = nullptr;
  hipStream_t s = nullptr;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  hipError_t alloc(nut_ctx *c, size_t bytes) {
    reset();
    s = c->stream;
    return hipMallocAsync(&p, bytes, s);
  }
  void reset() {
    if (p) (void)(s ? hipFreeAsync(p, s) : hipFree(p));
    p = nullptr;
  }
  ~DevBuf() { reset(); }
};
// what the programs of one nut_agg_spec point at: node arrays and LOOKUP tables (device)
struct ProgStore {
  std::deque<std::vector<nut_prog_node>> nodes;
  std::deque<DevBuf> tables;
};
// Key programs and countUnique arguments of a compiled aggregate plan, resolved against
// the spec's program columns (exec_groupby packs them into key words)
struct GbExtra {
  bool active = false;            // keys are programs: computed keys, > 2 keys or countUnique
  std::vector<int> slot;          // plan aggregate -> spec aggregate (-1: countUnique)
  std::vector<nut_prog> key;      // per GROUP BY key
  std::vector<nut_prog> cu_val, cu_mask;  // per plan aggregate (countUnique only)
};
// HAVING evaluation for group i: operands are int64 or f64 output words / constants;
// int-int comparisons are exact, anything else compares as f64
struct HVal {
  bool is_int;
  int64_t i;
  double f;
};
// NUT_COL_HOST columns: copied into stream-ordered HBM for one execute call
struct HostStage {
  std::vector<nut_column> cols;
  std::deque<DevBuf> bufs;
};

nut_status build_spec(const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts, uint64_t n,
                      nut_agg_spec &s, ProgStore &store, std::vector<int> &agg_f64, GbExtra *gx = nullptr);

// A plan column name inside EXISTS / IN subquery `scope` (>= 1): "\x1f<scope>\x1f<name>",
// so the same name in the outer query and in a subquery are two plan columns.
std::string scoped_name(int scope, sv name);
// the scope and bare name of a plan column name (scope 0: the outer query's)
int name_scope(const std::string &name, std::string *bare);

// ---- lower
bool ieq(sv a, sv b);
std::string i128_str(i128 v);
void json_str(std::string &o, sv s);
i128 sat_from_u128(u128 m, bool neg);
int64_t days_from_civil(int64_t y, unsigned m, unsigned d);
void civil_from_days(int64_t z, int64_t &y, unsigned &m, unsigned &d);
bool leap(int64_t y);
int64_t date_part(int64_t d, int part);
int date_fn(sv n);
unsigned month_days(int64_t y, unsigned m);
bool parse_date(sv s, int64_t &days);
int64_t add_months(int64_t days, i128 months);
bool const_eval(const Expr &e, CVal &out, Lowering &L);
std::string cval_str(const CVal &c);
i128 dec_floor(const Decimal &d, bool &frac);
int cmp_of(BinOp op);
int mirror(int op);
int pnode_arity(int op);
size_t u8len(const std::string &s, size_t i);
bool like_match(const std::string &str, const std::string &pat, bool ci);
int col_index(nut_plan &p, sv name);
bool column_ref(nut_plan &p, const Expr &e, sv &name);
std::string expr_text(const Expr &e);
bool is_one(const Expr &e);
bool lower_agg_expr(nut_plan &p, const Expr &e, PlanAgg &a, Lowering &L);
bool same_prog(const PProg &x, const PProg &y);
void emit(PProg &o, int op);
void emit_int(PProg &o, i128 v);
void emit_bool(PProg &o, bool b);
void append(PProg &o, const PProg &x);
int prog_binop(BinOp b);
bool is_null_lit(const Expr &e);
void bind_str(PProg &a, const PProg &other);
bool is_agg_name(sv n);
bool conditional(nut_plan &p, const Expr &e, std::vector<PProg> &conds, std::vector<const Expr *> &vals,
                 Lowering &L, bool &ok);
void chain(PProg &o, const std::vector<PProg> &conds, const std::vector<PProg> &vals);
bool lower_prog(nut_plan &p, const Expr &e, PProg &o, Lowering &L);
bool lower_nullable(nut_plan &p, const Expr &e, PProg &val, PProg &mask, bool &nullable, Lowering &L);
int add_agg(nut_plan &p, const PlanAgg &a);
bool lower_pred_term(nut_plan &p, const Expr &e, Lowering &L);
bool lower_where(nut_plan &p, const Expr &e, Lowering &L);
int key_of(nut_plan &p, const Expr &e);
bool is_distinct_name(sv n);
bool is_output_leaf(nut_plan &p, const Expr &e);
bool lower_xpr(nut_plan &p, const Expr &e, XNode &x, Lowering &L);
bool lower_output(nut_plan &p, const Expr &e, PlanOut &o, Lowering &L);
bool having_output(nut_plan &p, const Expr &e, int &out, Lowering &L);
bool lower_having(nut_plan &p, const Expr &e, HNode &h, Lowering &L);
bool on_equalities(nut_plan &p, const Expr &e, std::vector<std::pair<int, int>> &eqs);
bool add_key(nut_plan &p, const Expr &e, Lowering &L);
bool lower_mode(const Query &qry, nut_plan &p, Lowering &L);
bool resolve_using(nut_plan &p, Lowering &L);
bool lower_query(const Query &q, nut_plan &p, Lowering &L);
bool lower(const Statement &st, nut_plan &p, Lowering &L);
bool scalar_subquery(nut_plan &p, const Expr &e, CVal &c, Lowering &L);
std::string prog_text(const nut_plan &p, const PProg &pp);
std::string describe(const nut_plan &p);
nut_status put_text(const std::string &s, char *buf, size_t cap, size_t *len);
nut_status parse_into(const char *sql, size_t len, nut_stmt *s);

// ---- scan
Verdict resolve_i64(int op, const CVal &c, int &out_op, int64_t &k);
double resolve_f64(const CVal &c);
const nut_column *bind(const nut_plan &p, int ci, const nut_column *cols, int ncols);
bool needs_key_progs(const nut_plan &p);
nut_status topk_reduce(nut_ctx *c, const nut_plan &p, const void *keys, int type, bool desc, uint64_t n, DevBuf &pos,
                       uint64_t *m);
bool computed_proj(const nut_plan &p, size_t j);
nut_status exec_sort_rows(nut_ctx *c, const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts,
                          uint64_t n, nut_result *r);
enum ScanRoute { S_ROWID, S_RERUN_EXPR, S_EXPR_FILTER, S_EXPR_SORT, S_EXPR_SORT_F64, S_FUSED_FILTER, S_FUSED_SORT };
nut_status scan_route(const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts, ScanRoute *route);
const char *scan_route_name(ScanRoute r);
nut_status exec_scan(nut_ctx *c, const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts,
                     uint64_t n, nut_result *r);
HVal having_val(const HNode &h, const std::vector<std::vector<uint64_t>> &cols, const std::vector<int> &types,
                uint64_t g);
bool having_true(const HNode &h, const std::vector<std::vector<uint64_t>> &cols, const std::vector<int> &types,
                 uint64_t g);
nut_status check_strings(const nut_plan &p, const PProg &pp, const Dict *const *dicts, const char *what);
// the plan column whose dictionary decodes GROUP BY key j (a plain string column, or one
// substring of it), else -1
int key_dict_col(const nut_plan &p, size_t j);
// substring(s, off, len) with ClickHouse's byte semantics (P_SUBSTR)
std::string substr_bytes(const std::string &s, int off, i128 len);

// ---- groupby
nut_prog and_prog(const nut_prog &a, const nut_prog &b, ProgStore &store);
nut_status run_groupby(nut_ctx *c, const nut_agg_spec &s, uint64_t hint, std::vector<int64_t> &keys,
                       std::vector<uint64_t> &words, uint64_t &ng);
nut_status groupby_packed(nut_ctx *c, const nut_plan &p, const nut_agg_spec &s, const GbExtra &gx, ProgStore &store,
                          uint64_t hint, std::vector<int64_t> &keys, std::vector<uint64_t> &words, uint64_t &ng);
int xpr_type(const XNode &x, const std::vector<int> &types);
nut_status exec_groupby(nut_ctx *c, const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts,
                        uint64_t n, uint64_t hint, nut_result *r);

// ---- join
void split_and(const PProg &pp, std::vector<PProg> &out);
PProg and_all(const std::vector<PProg> &cs);
PProg pred_prog(const PlanPred &pr);
void add_null_mask(PlanAgg &a, int m);
bool mask_null_projections(nut_plan &q, const std::function<bool(int)> &nullable, const std::function<int(int)> &mflag);
const nut_plan *expand_star(const nut_plan &p, const std::vector<std::string> &names, nut_plan &q);
nut_status exec_join(nut_ctx *c, const nut_plan &p, const nut_column *lc, int nl, uint64_t lrows,
                     const nut_column *rc, int nr, uint64_t rrows, uint64_t hint, nut_result *r,
                     const Dict *const *ldict = nullptr, const Dict *const *rdict = nullptr);
nut_status exec_joinn(nut_ctx *c, const nut_plan &p, const nut_column *const *tabs, const int *ncols,
                      const uint64_t *nrows, int nt, uint64_t hint, nut_result *r,
                      const Dict *const *const *tdicts = nullptr);
nut_status stage_host(nut_ctx *c, const nut_column *cols, int n, uint64_t rows, HostStage &hs, const nut_column **out);

}  // namespace plan
}  // namespace nut
