// sql_plan.cpp — SQL C ABI (parse / tokenize / unescape) and plan lowering + execution
// (SURVEY.md §8(a) B1).
//
// The reference stops at the statement tree; what an executor lowers from is
//   QueryBody { columns, from, r#where, group_by, order_by, limit }  (ast/query.rs:21-35)
// with WHERE already constant-folded by the parser (simplify.rs), so a WHERE may arrive
// as a bare Literal::Boolean.  Lowering rules (DESIGN.md "Plan lowering"):
//   * WHERE: AND-chain of  col <cmp> const | const <cmp> col | col BETWEEN c1 AND c2 |
//     Boolean(true) (dropped) | Boolean(false) (empty result).  Comparisons are exact
//     in the column's type: against an int64 column a non-integral constant moves the
//     bound (x < 2.5 -> x <= 2) and an out-of-range constant folds to true/false.
//   * constants: Literal::Integer(u128, sign) and Literal::Float(BigDecimal) (exact,
//     converted with correct rounding for f64 columns), toDate('YYYY-MM-DD') and
//     date +/- interval n day|month|year, as days since 1970-01-01.
//   * SELECT-list FnCall Others(name): sum/count/min/max/avg, case-insensitive
//     (the parser keeps the original case, mod.rs:1305); count(*) is the wildcard
//     Identifier (mod.rs:1271); avg = sum / count.  Arguments: a column or one of the
//     fused expression shapes of nut_expr (a*b, a+b, a-b, a*(1-b), a*(1-b)*(1+c)).
//   * GROUP BY: 1-2 column identifiers; ORDER BY/LIMIT over the (small) group result
//     run on the host after the device aggregation.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <functional>
#include <memory>

#include "common.hpp"
#include "sql_ast.hpp"
#include "sort.hpp"
#include "sql_lexer.hpp"
#include "table.hpp"

using namespace nut;
using namespace nut::sql;

struct nut_stmt {
  std::string sql;   // the tree's views point into this copy
  Statement st;
};

namespace {

typedef __int128 i128;

bool ieq(sv a, sv b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i) {
    char x = a[i], y = b[i];
    if (x >= 'A' && x <= 'Z') x = (char)(x + 32);
    if (y >= 'A' && y <= 'Z') y = (char)(y + 32);
    if (x != y) return false;
  }
  return true;
}

std::string i128_str(i128 v) {
  if (v == 0) return "0";
  bool neg = v < 0;
  unsigned __int128 m = neg ? (unsigned __int128)(-(v + 1)) + 1 : (unsigned __int128)v;
  char buf[64];
  int i = 63;
  buf[i] = 0;
  while (m) {
    buf[--i] = (char)('0' + (int)(m % 10));
    m /= 10;
  }
  if (neg) buf[--i] = '-';
  return std::string(buf + i);
}

void json_str(std::string &o, sv s) {
  o += '"';
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += (char)c;
    } else if (c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      o += b;
    } else {
      o += (char)c;
    }
  }
  o += '"';
}

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

i128 sat_from_u128(u128 m, bool neg) {
  i128 v = m > (u128)kHuge ? kHuge : (i128)m;
  return neg ? -v : v;
}

// days since 1970-01-01 of a proleptic Gregorian date (civil-from-days inverse)
int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (int64_t)doe - 719468;
}
void civil_from_days(int64_t z, int64_t &y, unsigned &m, unsigned &d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const unsigned doe = (unsigned)(z - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  y = (int64_t)yoe + era * 400;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  d = doy - (153 * mp + 2) / 5 + 1;
  m = mp + (mp < 10 ? 3 : -9);
  y += m <= 2;
}
bool leap(int64_t y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }
// nut_date_part of a day number (the DATEPART program op's host twin, for constants)
int64_t date_part(int64_t d, int part) {
  d = std::max<int64_t>(-(1ll << 40), std::min<int64_t>(1ll << 40, d));
  int64_t y;
  unsigned m, dd;
  civil_from_days(d, y, m, dd);
  switch (part) {
    case NUT_DP_YEAR: return y;
    case NUT_DP_MONTH: return m;
    case NUT_DP_DAY: return dd;
    case NUT_DP_QUARTER: return (m - 1) / 3 + 1;
    case NUT_DP_WEEKDAY: return ((d % 7 + 7) % 7 + 3) % 7 + 1;
    case NUT_DP_YYYYMM: return y * 100 + m;
    case NUT_DP_YYYYMMDD: return y * 10000 + m * 100 + dd;
    default: return d - days_from_civil(y, 1, 1) + 1;
  }
}
// SQL date functions (ClickHouse names; getX spellings as in the reference's fixtures):
// the nut_date_part they compute, or -1
int date_fn(sv n) {
  static const char *const names[][2] = {{"toyear", "getyear"},         {"tomonth", "getmonth"},
                                          {"todayofmonth", "getdayofmonth"}, {"toquarter", "getquarter"},
                                          {"todayofweek", "getdayofweek"}, {"todayofyear", "getdayofyear"},
                                          {"toyyyymm", "toyyyymm"},         {"toyyyymmdd", "toyyyymmdd"}};
  for (int i = 0; i < 8; ++i)
    if (ieq(n, names[i][0]) || ieq(n, names[i][1])) return i;
  return -1;
}
unsigned month_days(int64_t y, unsigned m) {
  static const unsigned md[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  return m == 2 && leap(y) ? 29 : md[m - 1];
}

bool parse_date(sv s, int64_t &days) {
  if (s.size() != 10 || s[4] != '-' || s[7] != '-') return false;
  auto num = [&](size_t a, size_t n, int64_t &out) {
    out = 0;
    for (size_t i = a; i < a + n; ++i) {
      if (s[i] < '0' || s[i] > '9') return false;
      out = out * 10 + (s[i] - '0');
    }
    return true;
  };
  int64_t y, m, d;
  if (!num(0, 4, y) || !num(5, 2, m) || !num(8, 2, d)) return false;
  if (m < 1 || m > 12 || d < 1 || d > (int64_t)month_days(y, (unsigned)m)) return false;
  days = days_from_civil(y, (unsigned)m, (unsigned)d);
  return true;
}

// date +/- n months, clamping the day to the target month's length
int64_t add_months(int64_t days, i128 months) {
  int64_t y;
  unsigned m, d;
  civil_from_days(days, y, m, d);
  i128 t = (i128)y * 12 + (m - 1) + months;
  int64_t ny = (int64_t)(t >= 0 ? t / 12 : -((-t + 11) / 12));
  unsigned nm = (unsigned)(t - (i128)ny * 12) + 1;
  unsigned nd = std::min(d, month_days(ny, nm));
  return days_from_civil(ny, nm, nd);
}

struct Lowering {
  std::string err;
  bool fail(const std::string &m) {
    if (err.empty()) err = m;
    return false;
  }
};

bool const_eval(const Expr &e, CVal &out, Lowering &L) {
  if (e.k == EK::Literal) {
    const Literal &l = *e.lit;
    if (l.k == LitKind::Integer) {
      out.is_int = true;
      out.v = sat_from_u128(l.mag, !l.positive);
      return true;
    }
    if (l.k == LitKind::Float) {
      out.is_int = false;
      out.dec = l.dec;
      return true;
    }
    if (l.k == LitKind::String) {
      out.is_int = false;
      out.is_str = true;
      out.s = l.str;
      return true;
    }
    return false;
  }
  if (e.k == EK::FnCall && e.fn() == FnKind::Others && ieq(e.id.name, "todate") && e.kids.size() == 1 &&
      e.kids[0].k == EK::Literal && e.kids[0].lit->k == LitKind::String) {
    int64_t days;
    if (!parse_date(e.kids[0].lit->str, days)) return L.fail("toDate: '" + e.kids[0].lit->str + "' is not YYYY-MM-DD");
    out.is_int = true;
    out.v = days;
    return true;
  }
  if (e.k == EK::FnCall && e.fn() == FnKind::Others && date_fn(e.id.name) >= 0 && e.kids.size() == 1) {
    CVal x;
    if (!const_eval(e.kids[0], x, L) || !x.is_int || x.is_str) return false;
    out.is_int = true;
    out.v = date_part((int64_t)std::max<i128>(-(i128(1) << 41), std::min<i128>(i128(1) << 41, x.v)), date_fn(e.id.name));
    return true;
  }
  if (e.k == EK::BinaryOp && (e.bop() == BinOp::Plus || e.bop() == BinOp::Minus)) {
    const Expr &a = e.kids[0], &b = e.kids[1];
    const i128 sign = e.bop() == BinOp::Plus ? 1 : -1;
    CVal x;
    if (b.k == EK::Literal && b.lit->k == LitKind::Interval) {
      if (!const_eval(a, x, L) || !x.is_int) return false;
      const i128 n = sign * (i128)b.lit->interval;
      if (x.v > INT64_MAX || x.v < INT64_MIN) return false;
      switch (b.lit->unit) {
        case IntervalUnit::Day: out.v = x.v + n; break;
        case IntervalUnit::Month: out.v = add_months((int64_t)x.v, n); break;
        case IntervalUnit::Year: out.v = add_months((int64_t)x.v, 12 * n); break;
        default: return L.fail("interval units below a day do not apply to day-number columns");
      }
      out.is_int = true;
      return true;
    }
    CVal y;
    if (const_eval(a, x, L) && const_eval(b, y, L) && x.is_int && y.is_int) {
      i128 r = x.v + sign * y.v;
      out.is_int = true;
      out.v = r > kHuge ? kHuge : r < -kHuge ? -kHuge : r;
      return true;
    }
  }
  return false;
}

std::string cval_str(const CVal &c) {
  if (c.param >= 0) return "$subquery" + std::to_string(c.param);
  return c.is_str ? "'" + c.s + "'" : c.is_int ? i128_str(c.v) : c.dec.str();
}

// floor of an exact decimal, saturated; frac = true if it had a fractional part
i128 dec_floor(const Decimal &d, bool &frac) {
  const std::string &dg = d.digits;
  const int64_t sc = d.scale;
  const int64_t nint = (int64_t)dg.size() - sc;
  frac = false;
  i128 v = 0;
  for (int64_t i = 0; i < nint; ++i) {
    if (v > kHuge) break;
    v = v * 10 + (i < (int64_t)dg.size() ? dg[(size_t)i] - '0' : 0);
  }
  if (v > kHuge) v = kHuge;
  for (int64_t i = std::max<int64_t>(nint, 0); i < (int64_t)dg.size(); ++i)
    if (dg[(size_t)i] != '0') frac = true;
  if (d.neg) v = frac ? -v - 1 : -v;
  return v;
}

// ------------------------------------------------------------------ plan
const char *kCmpText[] = {"<", "<=", ">", ">=", "=", "!=", "in", "not in"};
int cmp_of(BinOp op) {
  switch (op) {
    case BinOp::Lt: return NUT_LT;
    case BinOp::LtEq: return NUT_LE;
    case BinOp::Gt: return NUT_GT;
    case BinOp::GtEq: return NUT_GE;
    case BinOp::Eq: return NUT_EQ;
    case BinOp::NotEq: return NUT_NE;
    default: return -1;
  }
}
int mirror(int op) { return op == NUT_LT ? NUT_GT : op == NUT_GT ? NUT_LT : op == NUT_LE ? NUT_GE : op == NUT_GE ? NUT_LE : op; }

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
  int arg = 0;   // NUT_P_DATEPART: nut_date_part
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

}  // namespace

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
    int key[2];
    int type = NUT_JOIN_INNER;  // NUT_JOIN_INNER / LEFT / SEMI / ANTI, PJ_RIGHT, PJ_FULL
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

namespace {

// internal program leaves (never reach nut_prog): `col [I]LIKE 'pattern'` over a
// dictionary column, lowered at execution to COL + LOOKUP in a per-code match table
constexpr int P_LIKE = 1000, P_ILIKE = 1001;

int pnode_arity(int op) {
  if (op == P_LIKE || op == P_ILIKE) return 0;
  return op <= NUT_P_F64 ? 0 : (op == NUT_P_NOT || op == NUT_P_BITNOT || op == NUT_P_ABS ||
                                op == NUT_P_TO_F64 || op == NUT_P_DATEPART) ? 1 : op == NUT_P_IF ? 3 : 2;
}

// bytes of the UTF-8 sequence starting at s[i] (a stray continuation byte counts alone)
size_t u8len(const std::string &s, size_t i) {
  const unsigned char c = (unsigned char)s[i];
  const size_t n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
  return std::min(n, s.size() - i);
}

// SQL LIKE: % any run, _ any one character (UTF-8 code point), backslash escapes the next
// pattern character; ILIKE folds ASCII case (other code points compare exactly)
bool like_match(const std::string &str, const std::string &pat, bool ci) {
  auto eq = [&](char a, char b) {
    if (ci) {
      a = (char)tolower((unsigned char)a);
      b = (char)tolower((unsigned char)b);
    }
    return a == b;
  };
  size_t s = 0, p = 0, star_p = std::string::npos, star_s = 0;
  while (s < str.size()) {
    if (p < pat.size() && pat[p] == '%') {
      star_p = ++p;
      star_s = s;
      continue;
    }
    if (p < pat.size()) {
      const bool esc = pat[p] == '\\' && p + 1 < pat.size();
      if (!esc && pat[p] == '_') {
        ++p;
        s += u8len(str, s);
        continue;
      }
      const size_t pp = esc ? p + 1 : p, pl = u8len(pat, pp), sl = u8len(str, s);
      bool same = pl == sl;
      for (size_t k = 0; same && k < pl; ++k) same = eq(pat[pp + k], str[s + k]);
      if (same) {
        p = pp + pl;
        s += sl;
        continue;
      }
    }
    if (star_p == std::string::npos) return false;
    p = star_p;
    star_s += u8len(str, star_s);
    s = star_s;
  }
  while (p < pat.size() && pat[p] == '%') ++p;
  return p == pat.size();
}

int col_index(nut_plan &p, sv name) {
  for (size_t i = 0; i < p.cols.size(); ++i)
    if (ieq(p.cols[i], name)) return (int)i;
  p.cols.emplace_back(name);
  return (int)p.cols.size() - 1;
}

// A column reference.  In a JOIN plan a qualified name keeps its qualifier ("o.custkey"):
// exec_join binds it to the table named or aliased so (and `a.k = b.k` can join two
// columns of the same name); elsewhere the qualifier is dropped.
bool column_ref(nut_plan &p, const Expr &e, sv &name) {
  if (e.k != EK::Identifier || e.id.wildcard) return false;
  if (p.join >= 0 && e.id.qualified) {
    p.qnames.push_back(std::string(e.id.qualifier) + "." + std::string(e.id.name));
    name = p.qnames.back();
  } else {
    name = e.id.name;
  }
  return true;
}

std::string expr_text(const Expr &e) {
  static const char *bin[] = {"+", "-", "*", "/", "%", ">", "<", ">=", "<=", "=", "!=", "and", "or",
                              "xor", "like", "not like", "ilike", "not ilike", "in", "not in", "[]",
                              "|", "&", "^", "<<", ">>"};
  switch (e.k) {
    case EK::Identifier: {
      std::string s;
      if (e.id.qualified) s = std::string(e.id.qualifier) + ".";
      return s + (e.id.wildcard ? std::string("*") : std::string(e.id.name));
    }
    case EK::Literal: {
      const Literal &l = *e.lit;
      if (l.k == LitKind::Integer) return (l.positive ? "" : "-") + i128_str((i128)l.mag);
      if (l.k == LitKind::Float) return l.dec.str();
      if (l.k == LitKind::String) return "'" + l.str + "'";
      if (l.k == LitKind::Boolean) return l.positive ? "true" : "false";
      return dump(e);
    }
    case EK::BinaryOp: {
      auto side = [](const Expr &x) {
        std::string t = expr_text(x);
        return x.k == EK::BinaryOp ? "(" + t + ")" : t;
      };
      return side(e.kids[0]) + " " + bin[e.op] + " " + side(e.kids[1]);
    }
    case EK::FnCall:
      if (e.fn() == FnKind::Others) {
        std::string s = std::string(e.id.name) + "(";
        for (size_t i = 0; i < e.kids.size(); ++i) s += (i ? ", " : "") + expr_text(e.kids[i]);
        return s + ")";
      }
      return dump(e);
    default: return dump(e);
  }
}

bool is_one(const Expr &e) {
  if (e.k != EK::Literal) return false;
  const Literal &l = *e.lit;
  if (l.k == LitKind::Integer) return l.positive && l.mag == 1;
  if (l.k == LitKind::Float) {
    Decimal one;
    one.digits = "1";
    return l.dec == one;
  }
  return false;
}

// SELECT-list aggregate argument -> fused expression shape (nut_expr)
bool lower_agg_expr(nut_plan &p, const Expr &e, PlanAgg &a, Lowering &L) {
  sv n0, n1, n2;
  auto val = [&](sv n) {
    int c = col_index(p, n);
    for (size_t i = 0; i < p.vals.size(); ++i)
      if (p.vals[i] == c) return (int)i;
    p.vals.push_back(c);
    return (int)p.vals.size() - 1;
  };
  a.arg[0] = a.arg[1] = a.arg[2] = 0;
  if (column_ref(p, e, n0)) {
    a.expr = NUT_EX_COL;
    a.arg[0] = val(n0);
    return true;
  }
  if (e.k == EK::BinaryOp) {
    const Expr &l = e.kids[0], &r = e.kids[1];
    if (column_ref(p, l, n0) && column_ref(p, r, n1)) {
      BinOp op = e.bop();
      if (op == BinOp::Multi || op == BinOp::Plus || op == BinOp::Minus) {
        a.expr = op == BinOp::Multi ? NUT_EX_MUL : op == BinOp::Plus ? NUT_EX_ADD : NUT_EX_SUB;
        a.arg[0] = val(n0);
        a.arg[1] = val(n1);
        return true;
      }
    }
    // a * (1 - b)
    if (e.bop() == BinOp::Multi && column_ref(p, l, n0) && r.k == EK::BinaryOp && r.bop() == BinOp::Minus &&
        is_one(r.kids[0]) && column_ref(p, r.kids[1], n1)) {
      a.expr = NUT_EX_MUL_1M;
      a.arg[0] = val(n0);
      a.arg[1] = val(n1);
      return true;
    }
    // a * (1 - b) * (1 + c)
    if (e.bop() == BinOp::Multi && l.k == EK::BinaryOp && l.bop() == BinOp::Multi && column_ref(p, l.kids[0], n0) &&
        l.kids[1].k == EK::BinaryOp && l.kids[1].bop() == BinOp::Minus && is_one(l.kids[1].kids[0]) &&
        column_ref(p, l.kids[1].kids[1], n1) && r.k == EK::BinaryOp && r.bop() == BinOp::Plus && is_one(r.kids[0]) &&
        column_ref(p, r.kids[1], n2)) {
      a.expr = NUT_EX_MUL_1M_1P;
      a.arg[0] = val(n0);
      a.arg[1] = val(n1);
      a.arg[2] = val(n2);
      return true;
    }
  }
  return L.fail("aggregate argument '" + expr_text(e) +
                "' is not a column or a fused expression shape (a*b, a+b, a-b, a*(1-b), a*(1-b)*(1+c))");
}

bool same_prog(const PProg &x, const PProg &y) {
  if (x.size() != y.size()) return false;
  for (size_t i = 0; i < x.size(); ++i) {
    const PNode &a = x[i], &b = y[i];
    if (a.op != b.op || a.col != b.col || a.arg != b.arg) return false;
    if (a.op == NUT_P_I64 && !(a.c.is_int == b.c.is_int && a.c.v == b.c.v && a.c.is_str == b.c.is_str &&
                               a.c.s == b.c.s))
      return false;
    if (a.op == NUT_P_F64 && !(a.c.dec == b.c.dec)) return false;
  }
  return true;
}

// ---- compiled mode: SQL expression -> RPN program (include/nutexec.h nut_prog_op)
void emit(PProg &o, int op) {
  PNode n;
  n.op = op;
  o.push_back(n);
}
void emit_int(PProg &o, i128 v) {
  PNode n;
  n.op = NUT_P_I64;
  n.c.is_int = true;
  n.c.v = v;
  o.push_back(n);
}
void emit_bool(PProg &o, bool b) {  // (b != 0): a bool-typed constant
  emit_int(o, b ? 1 : 0);
  emit_int(o, 0);
  emit(o, NUT_P_NE);
}
void append(PProg &o, const PProg &x) { o.insert(o.end(), x.begin(), x.end()); }

int prog_binop(BinOp b) {
  switch (b) {
    case BinOp::Plus: return NUT_P_ADD;
    case BinOp::Minus: return NUT_P_SUB;
    case BinOp::Multi: return NUT_P_MUL;
    case BinOp::Div: return NUT_P_DIV;
    case BinOp::Mod: return NUT_P_MOD;
    case BinOp::Gt: return NUT_P_GT;
    case BinOp::Lt: return NUT_P_LT;
    case BinOp::GtEq: return NUT_P_GE;
    case BinOp::LtEq: return NUT_P_LE;
    case BinOp::Eq: return NUT_P_EQ;
    case BinOp::NotEq: return NUT_P_NE;
    case BinOp::And: return NUT_P_AND;
    case BinOp::Or: return NUT_P_OR;
    case BinOp::Xor: return NUT_P_XOR;
    case BinOp::BitwiseOr: return NUT_P_BITOR;
    case BinOp::BitwiseAnd: return NUT_P_BITAND;
    case BinOp::BitwiseXor: return NUT_P_BITXOR;
    case BinOp::BitwiseLeftShift: return NUT_P_SHL;
    case BinOp::BitwiseRightShift: return NUT_P_SHR;
    default: return -1;
  }
}

bool is_null_lit(const Expr &e) { return e.k == EK::Literal && e.lit->k == LitKind::Null; }
// a string constant compared (= / != / IN / CASE x WHEN) with a column takes that
// column's dictionary at execution
void bind_str(PProg &a, const PProg &other) {
  if (a.size() == 1 && a[0].op == NUT_P_I64 && a[0].c.is_str && other.size() == 1 && other[0].op == NUT_P_COL)
    a[0].col = other[0].col;
}
bool is_agg_name(sv n) {
  return ieq(n, "sum") || ieq(n, "count") || ieq(n, "min") || ieq(n, "max") || ieq(n, "avg");
}

// A conditional: conds[i] -> vals[i], else vals.back().  CASE WHEN / IF / multiIf and
// CASE x WHEN v (cond x = v).  Returns false if e is not a conditional.
bool lower_prog(nut_plan &p, const Expr &e, PProg &o, Lowering &L);
bool scalar_subquery(nut_plan &p, const Expr &e, CVal &c, Lowering &L);
bool conditional(nut_plan &p, const Expr &e, std::vector<PProg> &conds, std::vector<const Expr *> &vals,
                 Lowering &L, bool &ok) {
  ok = true;
  if (e.k != EK::FnCall) return false;
  const FnKind f = e.fn();
  const bool fn_if = f == FnKind::Others && ieq(e.id.name, "if");
  const bool fn_multi = f == FnKind::Others && ieq(e.id.name, "multiif");
  if (f == FnKind::If || fn_if || f == FnKind::MultiIf || fn_multi) {
    const size_t n = e.kids.size();
    if ((f == FnKind::If || fn_if) ? n != 3 : (n < 3 || n % 2 == 0)) {
      ok = L.fail(std::string(fn_if ? "if" : "multiIf") + " takes a condition, a value and an else value" +
                  (fn_multi ? " (cond, value pairs, then else)" : ""));
      return true;
    }
    for (size_t i = 0; i + 1 < n; i += 2) {
      PProg c;
      if (!lower_prog(p, e.kids[i], c, L)) return ok = false, true;
      conds.push_back(std::move(c));
      vals.push_back(&e.kids[i + 1]);
    }
    vals.push_back(&e.kids[n - 1]);
    return true;
  }
  if (f == FnKind::CaseWhen) {
    const size_t n = e.kids.size();  // x, v1, a1, ..., else
    if (n < 4 || n % 2 != 0) return ok = L.fail("malformed CASE"), true;
    PProg x;
    if (!lower_prog(p, e.kids[0], x, L)) return ok = false, true;
    for (size_t i = 1; i + 1 < n; i += 2) {
      PProg c = x, v;
      if (!lower_prog(p, e.kids[i], v, L)) return ok = false, true;
      bind_str(v, x);
      append(c, v);
      emit(c, NUT_P_EQ);
      conds.push_back(std::move(c));
      vals.push_back(&e.kids[i + 1]);
    }
    vals.push_back(&e.kids[n - 1]);
    return true;
  }
  return false;
}
// c1 v1 c2 v2 ... else IF IF ... (IF pops cond, then, else)
void chain(PProg &o, const std::vector<PProg> &conds, const std::vector<PProg> &vals) {
  for (size_t i = 0; i < conds.size(); ++i) {
    append(o, conds[i]);
    append(o, vals[i]);
  }
  append(o, vals.back());
  for (size_t i = 0; i < conds.size(); ++i) emit(o, NUT_P_IF);
}

bool lower_prog(nut_plan &p, const Expr &e, PProg &o, Lowering &L) {
  CVal c;
  if (const_eval(e, c, L)) {
    PNode n;
    n.op = c.is_int || c.is_str ? NUT_P_I64 : NUT_P_F64;
    n.c = c;
    o.push_back(n);
    return true;
  }
  if (!L.err.empty()) return false;
  if (e.k == EK::Subquery) {
    PNode n;
    n.op = NUT_P_F64;  // the type is the subquery's, set when its value is put in
    if (!scalar_subquery(p, e, n.c, L)) return L.fail(L.err.empty() ? "subquery is not a value here" : L.err);
    o.push_back(n);
    return true;
  }
  switch (e.k) {
    case EK::Identifier: {
      if (e.id.wildcard) return L.fail("'*' is not a value");
      PNode n;
      n.op = NUT_P_COL;
      sv nm;
      column_ref(p, e, nm);
      n.col = col_index(p, nm);
      o.push_back(n);
      return true;
    }
    case EK::Literal: {
      bool b;
      if (e.is_bool_lit(&b)) {
        emit_bool(o, b);
        return true;
      }
      if (is_null_lit(e)) return L.fail("NULL is executed only as a CASE/IF branch of an aggregate argument");
      return L.fail("literal '" + expr_text(e) + "' is not executed here");
    }
    case EK::BinaryOp: {
      const BinOp b = e.bop();
      if (b == BinOp::In || b == BinOp::NotIn) {
        const bool in = b == BinOp::In;
        const Expr &r = e.kids[1];
        if (r.k == EK::Subquery) return L.fail("IN (subquery) is not executed");
        std::vector<const Expr *> items;
        if (r.k == EK::Collection && (CollType)r.op == CollType::Tuple)
          for (const Expr &x : r.kids) items.push_back(&x);
        else
          items.push_back(&r);
        if (items.empty()) {
          emit_bool(o, !in);
          return true;
        }
        PProg x;
        if (!lower_prog(p, e.kids[0], x, L)) return false;
        for (size_t i = 0; i < items.size(); ++i) {
          append(o, x);
          PProg it;
          if (!lower_prog(p, *items[i], it, L)) return false;
          bind_str(it, x);
          append(o, it);
          emit(o, in ? NUT_P_EQ : NUT_P_NE);
          if (i) emit(o, in ? NUT_P_OR : NUT_P_AND);
        }
        return true;
      }
      if (b == BinOp::Like || b == BinOp::NotLike || b == BinOp::ILike || b == BinOp::NotILike) {
        sv cname;
        CVal pat;
        if (!column_ref(p, e.kids[0], cname) || !const_eval(e.kids[1], pat, L) || !pat.is_str)
          return L.fail("LIKE takes a column and a string pattern ('" + expr_text(e) + "')");
        PNode n;
        n.op = (b == BinOp::ILike || b == BinOp::NotILike) ? P_ILIKE : P_LIKE;
        n.col = col_index(p, cname);
        n.c = pat;
        o.push_back(n);
        if (b == BinOp::NotLike || b == BinOp::NotILike) emit(o, NUT_P_NOT);
        return true;
      }
      const int op = prog_binop(b);
      if (op < 0) return L.fail("operator in '" + expr_text(e) + "' is not executed ([] and friends)");
      PProg l, r;
      if (!lower_prog(p, e.kids[0], l, L) || !lower_prog(p, e.kids[1], r, L)) return false;
      if (op == NUT_P_EQ || op == NUT_P_NE) {
        bind_str(l, r);
        bind_str(r, l);
      }
      append(o, l);
      append(o, r);
      emit(o, op);
      return true;
    }
    case EK::UnaryOp: {
      const UnOp u = e.uop();
      if (u == UnOp::IsNull || u == UnOp::IsNotNull) {  // executed columns hold no NULLs
        PProg tmp;
        if (!lower_prog(p, e.kids[0], tmp, L)) return false;
        for (const PNode &nd : tmp)  // (a NULL-extended table's column would: joins reject it)
          if (nd.op == NUT_P_COL) p.isnull_cols.push_back(nd.col);
        emit_bool(o, u == UnOp::IsNotNull);
        return true;
      }
      if (!lower_prog(p, e.kids[0], o, L)) return false;
      emit(o, u == UnOp::Not ? NUT_P_NOT : NUT_P_BITNOT);
      return true;
    }
    case EK::FnCall: {
      std::vector<PProg> conds;
      std::vector<const Expr *> vals;
      bool ok;
      if (conditional(p, e, conds, vals, L, ok)) {
        if (!ok) return false;
        std::vector<PProg> vp(vals.size());
        for (size_t i = 0; i < vals.size(); ++i)
          if (!lower_prog(p, *vals[i], vp[i], L)) return false;
        chain(o, conds, vp);
        return true;
      }
      const FnKind f = e.fn();
      if (f == FnKind::Between || f == FnKind::NotBetween) {
        if (e.kids.size() != 3) return L.fail("malformed BETWEEN");
        const bool in = f == FnKind::Between;
        for (int side = 0; side < 2; ++side) {
          if (!lower_prog(p, e.kids[0], o, L) || !lower_prog(p, e.kids[1 + side], o, L)) return false;
          emit(o, side == 0 ? (in ? NUT_P_GE : NUT_P_LT) : (in ? NUT_P_LE : NUT_P_GT));
        }
        emit(o, in ? NUT_P_AND : NUT_P_OR);
        return true;
      }
      if (f != FnKind::Others) return L.fail("'" + expr_text(e) + "' (EXISTS / subqueries) is not executed");
      const sv n = e.id.name;
      const size_t na = e.kids.size();
      if (is_agg_name(n)) return L.fail("aggregate '" + std::string(n) + "' nested inside an expression");
      if ((ieq(n, "abs") || ieq(n, "tofloat64")) && na == 1) {
        if (!lower_prog(p, e.kids[0], o, L)) return false;
        emit(o, ieq(n, "abs") ? NUT_P_ABS : NUT_P_TO_F64);
        return true;
      }
      if ((ieq(n, "intdiv") || ieq(n, "modulo")) && na == 2) {
        if (!lower_prog(p, e.kids[0], o, L) || !lower_prog(p, e.kids[1], o, L)) return false;
        emit(o, ieq(n, "intdiv") ? NUT_P_INTDIV : NUT_P_MOD);
        return true;
      }
      if (date_fn(n) >= 0 && na == 1) {
        if (!lower_prog(p, e.kids[0], o, L)) return false;
        PNode dp;
        dp.op = NUT_P_DATEPART;
        dp.arg = date_fn(n);
        o.push_back(dp);
        return true;
      }
      if (ieq(n, "todate")) return L.fail("toDate takes one 'YYYY-MM-DD' constant");
      return L.fail("function '" + std::string(n) + "' is not executed (executed: if, multiIf, abs, toFloat64, intDiv, "
                    "modulo, toYear/getYear, toMonth, toDayOfMonth, toQuarter, toDayOfWeek, toDayOfYear, toYYYYMM, "
                    "toYYYYMMDD)");
    }
    default: return L.fail("'" + expr_text(e) + "' is not executed (parameters, collections, subqueries)");
  }
}

// An aggregate argument: a NULL branch of a top-level conditional (CASE without ELSE)
// becomes the aggregate's row mask — SQL aggregates skip NULL arguments.
bool lower_nullable(nut_plan &p, const Expr &e, PProg &val, PProg &mask, bool &nullable, Lowering &L) {
  nullable = false;
  if (is_null_lit(e)) {
    emit_int(val, 0);
    emit_bool(mask, false);
    nullable = true;
    return true;
  }
  std::vector<PProg> conds;
  std::vector<const Expr *> vals;
  bool ok;
  if (!conditional(p, e, conds, vals, L, ok)) return lower_prog(p, e, val, L);
  if (!ok) return false;
  std::vector<PProg> vv(vals.size()), mm(vals.size());
  std::vector<char> nb(vals.size());
  for (size_t i = 0; i < vals.size(); ++i) {
    bool n;
    if (!lower_nullable(p, *vals[i], vv[i], mm[i], n, L)) return false;
    nb[i] = n;
    nullable = nullable || n;
  }
  chain(val, conds, vv);
  if (nullable) {
    for (size_t i = 0; i < vals.size(); ++i)
      if (!nb[i]) emit_bool(mm[i], true);
    chain(mask, conds, mm);
  }
  return true;
}

int add_agg(nut_plan &p, const PlanAgg &a) {
  // count(x) and count(*) differ only once an outer join masks x's table
  bool outer = p.join == NUT_JOIN_LEFT || p.join == PJ_FULL;
  for (const nut_plan::JoinStep &js : p.jn)
    outer = outer || js.type == NUT_JOIN_LEFT || js.type == PJ_RIGHT || js.type == PJ_FULL;
  for (size_t i = 0; i < p.aggs.size(); ++i) {
    const PlanAgg &b = p.aggs[i];
    if (p.compiled) {
      if (b.op == a.op && b.distinct == a.distinct && same_prog(b.mask, a.mask) &&
          (a.op == NUT_AGG_COUNT || same_prog(b.val, a.val)) && (!a.distinct || same_prog(b.val, a.val)) &&
          (b.refs == a.refs || (a.op == NUT_AGG_COUNT && !a.distinct && !outer)))
        return (int)i;
      continue;
    }
    if (b.op == a.op && (a.op == NUT_AGG_COUNT ||
                         (b.expr == a.expr && !memcmp(b.arg, a.arg, sizeof a.arg))))
      return (int)i;
  }
  p.aggs.push_back(a);
  return (int)p.aggs.size() - 1;
}

bool lower_pred_term(nut_plan &p, const Expr &e, Lowering &L) {
  bool b;
  if (e.is_bool_lit(&b)) {
    if (!b) p.never = true;
    return true;
  }
  sv name;
  CVal c;
  if (e.k == EK::BinaryOp && cmp_of(e.bop()) >= 0) {
    int op = cmp_of(e.bop());
    const Expr &l = e.kids[0], &r = e.kids[1];
    if (column_ref(p, l, name) && (const_eval(r, c, L) || scalar_subquery(p, r, c, L))) {
      p.preds.push_back({col_index(p, name), op, c});
      return true;
    }
    if (column_ref(p, r, name) && (const_eval(l, c, L) || scalar_subquery(p, l, c, L))) {
      p.preds.push_back({col_index(p, name), mirror(op), c});
      return true;
    }
    if (!L.err.empty()) return false;
  }
  if (e.k == EK::BinaryOp && (e.bop() == BinOp::In || e.bop() == BinOp::NotIn) && column_ref(p, e.kids[0], name)) {
    // col [NOT] IN (c1, c2, ...): a tuple of constants, or one constant
    const Expr &r = e.kids[1];
    PlanPred pr{col_index(p, name), e.bop() == BinOp::In ? NUT_IN : NUT_NOT_IN, CVal{}, {}};
    if (r.k == EK::Collection && (CollType)r.op == CollType::Tuple) {
      for (const Expr &x : r.kids) {
        CVal v;
        if (!const_eval(x, v, L)) return L.fail("IN list item '" + expr_text(x) + "' is not a constant");
        pr.set.push_back(v);
      }
    } else {
      CVal v;
      if (!const_eval(r, v, L)) return L.fail("IN needs a list of constants (subqueries are not executed)");
      pr.set.push_back(v);
    }
    if (pr.set.size() > NUT_MAX_SET) return L.fail("IN lists hold at most 16 values");
    p.preds.push_back(std::move(pr));
    return true;
  }
  if (e.k == EK::FnCall && e.fn() == FnKind::Between && e.kids.size() == 3 && column_ref(p, e.kids[0], name)) {
    CVal lo, hi;
    if (const_eval(e.kids[1], lo, L) && const_eval(e.kids[2], hi, L)) {
      int ci = col_index(p, name);
      p.preds.push_back({ci, NUT_GE, lo});
      p.preds.push_back({ci, NUT_LE, hi});
      return true;
    }
  }
  return L.fail("unsupported WHERE term '" + expr_text(e) + "' (expected column <cmp> constant)");
}

bool lower_where(nut_plan &p, const Expr &e, Lowering &L) {
  if (e.k == EK::BinaryOp && e.bop() == BinOp::And)
    return lower_where(p, e.kids[0], L) && lower_where(p, e.kids[1], L);
  return lower_pred_term(p, e, L);
}

// the GROUP BY key an expression names (its column, or a computed key's text), or -1
int key_of(nut_plan &p, const Expr &e) {
  sv name;
  if (column_ref(p, e, name)) {
    const int c = col_index(p, name);
    for (size_t i = 0; i < p.keys.size(); ++i)
      if (p.keys[i] == c) return (int)i;
    return -1;
  }
  const std::string t = expr_text(e);
  for (size_t i = 0; i < p.key_text.size(); ++i)
    if (p.keys[i] < 0 && ieq(p.key_text[i], t)) return (int)i;
  return -1;
}
bool is_distinct_name(sv n) { return ieq(n, "countunique") || ieq(n, "uniqexact") || ieq(n, "uniq"); }
bool is_output_leaf(nut_plan &p, const Expr &e) {
  return key_of(p, e) >= 0 ||
         (e.k == EK::FnCall && e.fn() == FnKind::Others && (is_agg_name(e.id.name) || is_distinct_name(e.id.name)));
}
bool having_output(nut_plan &p, const Expr &e, int &out, Lowering &L);

// arithmetic over keys / aggregates / constants (an OUT_EXPR output)
bool lower_xpr(nut_plan &p, const Expr &e, XNode &x, Lowering &L) {
  CVal c;
  Lowering quiet;
  if (const_eval(e, c, quiet)) {
    if (c.is_str) return L.fail("string constants in arithmetic over aggregates are not executed");
    x.k = X_CONST;
    if (c.is_int && c.v <= INT64_MAX && c.v >= INT64_MIN) {
      x.is_int = true;
      x.i = (int64_t)c.v;
    } else {
      x.is_int = false;
      x.f = c.is_int ? (double)c.v : c.dec.to_f64();
    }
    return true;
  }
  if (is_output_leaf(p, e)) {
    x.k = X_OUT;
    return having_output(p, e, x.out, L);
  }
  if (e.k == EK::BinaryOp) {
    const BinOp b = e.bop();
    const int k = b == BinOp::Plus ? X_ADD : b == BinOp::Minus ? X_SUB : b == BinOp::Multi ? X_MUL
                  : b == BinOp::Div ? X_DIV : b == BinOp::Mod ? X_MOD : -1;
    if (k < 0) return L.fail("operator in '" + expr_text(e) + "' is not executed over aggregates (+ - * / %)");
    x.k = k;
    x.kids.resize(2);
    return lower_xpr(p, e.kids[0], x.kids[0], L) && lower_xpr(p, e.kids[1], x.kids[1], L);
  }
  if (e.k == EK::FnCall && e.fn() == FnKind::Others) {
    const sv n = e.id.name;
    const size_t na = e.kids.size();
    int k = -1;
    if ((ieq(n, "intdiv") || ieq(n, "modulo")) && na == 2) k = ieq(n, "intdiv") ? X_INTDIV : X_MOD;
    if ((ieq(n, "abs") || ieq(n, "tofloat64")) && na == 1) k = ieq(n, "abs") ? X_ABS : X_TOF;
    if (k >= 0) {
      x.k = k;
      x.kids.resize(na);
      for (size_t i = 0; i < na; ++i)
        if (!lower_xpr(p, e.kids[i], x.kids[i], L)) return false;
      return true;
    }
  }
  return L.fail("SELECT item '" + expr_text(e) + "' is not a GROUP BY key, an aggregate or arithmetic over them");
}

// one SELECT-list item of an aggregate plan: a GROUP BY key, sum/count/min/max/avg,
// countUnique, or arithmetic over those
bool lower_output(nut_plan &p, const Expr &e, PlanOut &o, Lowering &L) {
  sv name;
  const int kj = key_of(p, e);
  if (kj >= 0) {
    o.kind = OUT_KEY;
    o.a = kj;
    return true;
  }
  if (column_ref(p, e, name))
    return L.fail("column '" + std::string(name) + "' is neither a GROUP BY key nor aggregated" +
                  (p.keys.empty() ? " (no GROUP BY)" : ""));
  if (!(e.k == EK::FnCall && e.fn() == FnKind::Others && (is_agg_name(e.id.name) || is_distinct_name(e.id.name)))) {
    XNode x;
    if (!lower_xpr(p, e, x, L)) return false;
    p.xprs.push_back(std::move(x));
    o.kind = OUT_EXPR;
    o.a = (int)p.xprs.size() - 1;
    return true;
  }
  sv fn = e.id.name;
  if (is_distinct_name(fn)) {
    // countUnique(x): distinct x per group — GROUP BY (keys, x), then a count per key
    // tuple (exec_groupby); expression mode only
    if (!p.compiled) return L.fail("countUnique runs in expression mode");
    if (e.kids.size() != 1) return L.fail(std::string(fn) + " takes one argument");
    PlanAgg a{};
    bool nullable = false;
    if (!lower_nullable(p, e.kids[0], a.val, a.mask, nullable, L)) return false;
    for (const PProg *pp : {&a.val, &a.mask})
      for (const PNode &nd : *pp)
        if (nd.op == NUT_P_COL || nd.op == P_LIKE || nd.op == P_ILIKE) a.refs.push_back(nd.col);
    std::sort(a.refs.begin(), a.refs.end());
    a.refs.erase(std::unique(a.refs.begin(), a.refs.end()), a.refs.end());
    a.op = NUT_AGG_COUNT;
    a.expr = NUT_EX_COL;
    a.distinct = true;
    o.kind = OUT_AGG;
    o.a = add_agg(p, a);
    return true;
  }
  int op = ieq(fn, "sum") ? NUT_AGG_SUM : ieq(fn, "count") ? NUT_AGG_COUNT : ieq(fn, "min") ? NUT_AGG_MIN
           : ieq(fn, "max") ? NUT_AGG_MAX : ieq(fn, "avg") ? 100 : -1;
  if (op < 0) return L.fail("function '" + std::string(fn) + "' is not an executed aggregate (sum/count/min/max/avg)");
  PlanAgg a{};
  if (p.compiled) {
    if (op == NUT_AGG_COUNT ? e.kids.size() > 1 : e.kids.size() != 1)
      return L.fail(std::string(fn) + (op == NUT_AGG_COUNT ? " takes at most one argument" : " takes one argument"));
    bool nullable = false;
    const bool star = e.kids.empty() || (e.kids[0].k == EK::Identifier && e.kids[0].id.wildcard);
    if (!star && !lower_nullable(p, e.kids[0], a.val, a.mask, nullable, L)) return false;
    for (const PProg *pp : {&a.val, &a.mask})
      for (const PNode &nd : *pp)
        if (nd.op == NUT_P_COL || nd.op == P_LIKE || nd.op == P_ILIKE) a.refs.push_back(nd.col);
    std::sort(a.refs.begin(), a.refs.end());
    a.refs.erase(std::unique(a.refs.begin(), a.refs.end()), a.refs.end());
    if (op == NUT_AGG_COUNT) a.val.clear();  // count(x) counts the rows where x is not NULL
    a.op = op == 100 ? NUT_AGG_SUM : op;
    a.expr = NUT_EX_COL;
    o.a = add_agg(p, a);
    o.kind = op == 100 ? OUT_AVG : OUT_AGG;
    if (op == 100) {
      PlanAgg cnt{};
      cnt.op = NUT_AGG_COUNT;
      cnt.expr = NUT_EX_COL;
      cnt.mask = a.mask;
      cnt.refs = a.refs;
      o.b = add_agg(p, cnt);
    }
    return true;
  }
  if (op == NUT_AGG_COUNT) {
    if (e.kids.size() > 1) return L.fail("count takes at most one argument");
    if (e.kids.size() == 1 && !(e.kids[0].k == EK::Identifier)) return L.fail("count argument must be * or a column");
    a.op = NUT_AGG_COUNT;
    a.expr = NUT_EX_COL;
    o.kind = OUT_AGG;
    o.a = add_agg(p, a);
    return true;
  }
  if (e.kids.size() != 1) return L.fail(std::string(fn) + " takes one argument");
  if (!lower_agg_expr(p, e.kids[0], a, L)) return false;
  if (op == 100) {
    a.op = NUT_AGG_SUM;
    o.kind = OUT_AVG;
    o.a = add_agg(p, a);
    PlanAgg c{};
    c.op = NUT_AGG_COUNT;
    o.b = add_agg(p, c);
  } else {
    a.op = op;
    o.kind = OUT_AGG;
    o.a = add_agg(p, a);
  }
  return true;
}

// an output for a HAVING operand: reuse a SELECT item with the same text, else add a
// hidden one
bool having_output(nut_plan &p, const Expr &e, int &out, Lowering &L) {
  const std::string text = expr_text(e);
  for (size_t i = 0; i < p.outs.size(); ++i)
    if (ieq(p.outs[i].text, text) || (!p.outs[i].hidden && ieq(p.outs[i].name, text))) {
      out = (int)i;
      return true;
    }
  PlanOut o;
  o.text = o.name = text;
  o.hidden = true;
  if (!lower_output(p, e, o, L)) return false;
  p.outs.push_back(std::move(o));
  out = (int)p.outs.size() - 1;
  return true;
}

// HAVING: AND/OR/NOT of comparisons between aggregates, keys and constants
bool lower_having(nut_plan &p, const Expr &e, HNode &h, Lowering &L) {
  bool bv;
  if (e.is_bool_lit(&bv)) {
    h.k = H_BOOL;
    h.b = bv;
    return true;
  }
  if (e.k == EK::UnaryOp && e.uop() == UnOp::Not) {
    h.k = H_NOT;
    h.kids.resize(1);
    return lower_having(p, e.kids[0], h.kids[0], L);
  }
  if (e.k == EK::BinaryOp && (e.bop() == BinOp::And || e.bop() == BinOp::Or)) {
    h.k = e.bop() == BinOp::And ? H_AND : H_OR;
    h.kids.resize(2);
    return lower_having(p, e.kids[0], h.kids[0], L) && lower_having(p, e.kids[1], h.kids[1], L);
  }
  auto operand = [&](const Expr &x, HNode &o) {
    CVal c;
    Lowering quiet;
    if (x.k == EK::Subquery) {
      if (!scalar_subquery(p, x, c, L)) return false;
      o.k = H_CONST;
      o.param = c.param;
      return true;
    }
    if (const_eval(x, c, quiet)) {
      if (c.is_str) return L.fail("string constants in HAVING are not executed");
      o.k = H_CONST;
      if (c.is_int && c.v <= INT64_MAX && c.v >= INT64_MIN) {
        o.is_int = true;
        o.i = (int64_t)c.v;
      } else {
        o.f = c.is_int ? (double)c.v : c.dec.to_f64();
      }
      return true;
    }
    o.k = H_OUT;
    return having_output(p, x, o.out, L);
  };
  if (e.k == EK::BinaryOp && cmp_of(e.bop()) >= 0) {
    h.k = H_CMP;
    h.op = cmp_of(e.bop());
    h.kids.resize(2);
    return operand(e.kids[0], h.kids[0]) && operand(e.kids[1], h.kids[1]);
  }
  if (e.k == EK::FnCall && (e.fn() == FnKind::Between || e.fn() == FnKind::NotBetween) && e.kids.size() == 3) {
    HNode lo, hi, x;
    if (!operand(e.kids[0], x) || !operand(e.kids[1], lo) || !operand(e.kids[2], hi)) return false;
    HNode ge, le;
    ge.k = le.k = H_CMP;
    ge.op = NUT_GE;
    le.op = NUT_LE;
    ge.kids = {x, lo};
    le.kids = {x, hi};
    HNode both;
    both.k = H_AND;
    both.kids = {ge, le};
    if (e.fn() == FnKind::Between) {
      h = std::move(both);
    } else {
      h.k = H_NOT;
      h.kids = {both};
    }
    return true;
  }
  return L.fail("unsupported HAVING term '" + expr_text(e) + "'");
}

PProg and_all(const std::vector<PProg> &cs);

// ON a = b [AND c = d ...]: every equality of two columns, in order (the first is the hash
// key, the rest residual equalities); false if the condition has any other shape
bool on_equalities(nut_plan &p, const Expr &e, std::vector<std::pair<int, int>> &eqs) {
  if (e.k == EK::BinaryOp && e.bop() == BinOp::And)
    return on_equalities(p, e.kids[0], eqs) && on_equalities(p, e.kids[1], eqs);
  sv ka, kb;
  if (!(e.k == EK::BinaryOp && e.bop() == BinOp::Eq && column_ref(p, e.kids[0], ka) && column_ref(p, e.kids[1], kb)))
    return false;
  const int a = col_index(p, ka);
  eqs.emplace_back(a, col_index(p, kb));
  return true;
}

// one GROUP BY key: a column (fused and expression mode) or, in expression mode, any
// integer expression (getYear(d), a % 10, ...) evaluated by the group-by kernel
bool add_key(nut_plan &p, const Expr &e, Lowering &L) {
  sv name;
  PProg kp;
  if (column_ref(p, e, name)) {
    const int c = col_index(p, name);
    for (int k : p.keys)
      if (k == c) return true;  // GROUP BY a, a: one key
    p.keys.push_back(c);
    PNode n;
    n.op = NUT_P_COL;
    n.col = c;
    kp.push_back(n);
  } else {
    if (!p.compiled) return L.fail("computed GROUP BY keys run in expression mode");
    if (!lower_prog(p, e, kp, L)) return false;
    p.keys.push_back(-1);
  }
  p.key_progs.push_back(std::move(kp));
  p.key_text.push_back(expr_text(e));
  return true;
}

bool lower_mode(const Query &qry, nut_plan &p, Lowering &L) {
  if (qry.is_union) return L.fail("UNION/INTERSECT/EXCEPT are not executed (one query body per plan)");
  const QueryBody &b = *qry.body;
  if (b.with) return L.fail("WITH is not executed");
  if (b.distinct && b.group_by) return L.fail("DISTINCT with GROUP BY is not executed");
  if (!b.from || b.from->k != SourceKind::Table) return L.fail("FROM must name one table");
  std::vector<std::pair<int, int>> join_extra;  // residual ON equalities (INNER), applied as WHERE terms
  if (b.joins.size() > 1) {  // a chain of INNER / LEFT joins: FROM t0 JOIN t1 ON .. LEFT JOIN t2 ON ..
    p.join = NUT_JOIN_INNER;
    if (b.from->alias) p.talias = std::string(*b.from->alias);
    for (const JoinClause &jc : b.joins) {
      if (jc.src.k != SourceKind::Table) return L.fail("JOIN source must be a table");
      if (!jc.on) return L.fail("JOIN ... USING in a chain of joins is not executed (ON a = b)");
      int type;
      switch (jc.t) {
        case JoinType::Inner: type = NUT_JOIN_INNER; break;
        case JoinType::LeftOuter: type = NUT_JOIN_LEFT; break;
        case JoinType::RightOuter: type = PJ_RIGHT; break;
        case JoinType::FullOuter: type = PJ_FULL; break;
        case JoinType::LeftSemi: type = NUT_JOIN_SEMI; break;
        case JoinType::LeftAnti: type = NUT_JOIN_ANTI; break;
        default: return L.fail("several JOINs: INNER, LEFT / RIGHT / FULL OUTER, LEFT SEMI / ANTI steps only");
      }
      std::vector<std::pair<int, int>> eqs;
      if (!on_equalities(p, jc.cond, eqs))
        return L.fail("JOIN ON must be equalities of two columns (ANDed)");
      if (eqs.size() > 1 && jc.t != JoinType::Inner)
        return L.fail("JOIN with several key columns: INNER only (outer / semi / anti joins take one ON equality)");
      nut_plan::JoinStep js;
      js.type = type;
      js.table = std::string(jc.src.table);
      if (jc.src.alias) js.alias = std::string(*jc.src.alias);
      js.key[0] = eqs[0].first;
      js.key[1] = eqs[0].second;
      p.jn.push_back(js);
      join_extra.insert(join_extra.end(), eqs.begin() + 1, eqs.end());
    }
    if (p.jn.size() > 15) return L.fail("at most 16 joined tables");
    p.jtable = p.jn[0].table;
    p.jalias = p.jn[0].alias;
    p.jkey[0] = p.jn[0].key[0];
    p.jkey[1] = p.jn[0].key[1];
  } else if (!b.joins.empty()) {
    const JoinClause &jc = b.joins[0];
    if (jc.src.k != SourceKind::Table) return L.fail("JOIN source must be a table");
    switch (jc.t) {
      case JoinType::Inner: p.join = NUT_JOIN_INNER; break;
      case JoinType::LeftOuter: p.join = NUT_JOIN_LEFT; break;
      case JoinType::RightOuter: p.join = NUT_JOIN_LEFT, p.jright = true; break;
      case JoinType::LeftSemi: p.join = NUT_JOIN_SEMI; break;
      case JoinType::RightSemi: p.join = NUT_JOIN_SEMI, p.jright = true; break;
      case JoinType::LeftAnti: p.join = NUT_JOIN_ANTI; break;
      case JoinType::RightAnti: p.join = NUT_JOIN_ANTI, p.jright = true; break;
      case JoinType::FullOuter: p.join = PJ_FULL; break;
      default: return L.fail("ASOF JOIN is not executed");
    }
    p.jtable = std::string(jc.src.table);
    if (jc.src.alias) p.jalias = std::string(*jc.src.alias);
    if (b.from && b.from->alias) p.talias = std::string(*b.from->alias);
    std::vector<std::pair<int, int>> eqs;  // (p.join is set: qualified ON columns keep their qualifier)
    if (jc.on) {
      if (!on_equalities(p, jc.cond, eqs)) return L.fail("JOIN ON must be equalities of two columns (ANDed)");
    } else {
      // USING (u, ...): u of the FROM table = u of the JOIN source; an unqualified u
      // elsewhere in the query is the preserved table's (INNER: the FROM table's)
      const std::string lq = p.talias.empty() ? std::string(b.from->table) : p.talias;
      const std::string rq = p.jalias.empty() ? p.jtable : p.jalias;
      for (const Identifier &u : jc.using_) {
        const std::string un(u.name);
        eqs.emplace_back(col_index(p, p.qnames.emplace_back(lq + "." + un)),
                         col_index(p, p.qnames.emplace_back(rq + "." + un)));
        p.using_cols.push_back({un, p.jright ? rq + "." + un : lq + "." + un});
      }
      if (eqs.empty()) return L.fail("JOIN ... USING () names no column");
    }
    if (eqs.size() > 1 && p.join != NUT_JOIN_INNER)
      return L.fail("JOIN with several key columns: INNER only (outer / semi / anti joins take one ON equality)");
    p.jkey[0] = eqs[0].first;
    p.jkey[1] = eqs[0].second;
    join_extra.insert(join_extra.end(), eqs.begin() + 1, eqs.end());
  }
  if (b.having && !b.group_by) return L.fail("HAVING needs GROUP BY");
  p.table = std::string(b.from->table);
  bool wb;
  if (p.compiled && b.where) {
    if (b.where->is_bool_lit(&wb)) {
      if (!wb) p.never = true;
    } else if (!lower_prog(p, *b.where, p.where, L)) {
      return false;
    }
  } else if (b.where && !lower_where(p, *b.where, L)) {
    return false;
  }
  if (!join_extra.empty()) {  // the further key columns of the join: equalities above it
    if (!p.compiled) return L.fail("JOIN with several key columns runs in expression mode");
    std::vector<PProg> cs;
    if (!p.where.empty()) cs.push_back(p.where);
    for (const auto &e : join_extra) {
      PNode a, c, eq;
      a.op = NUT_P_COL;
      a.col = e.first;
      c.op = NUT_P_COL;
      c.col = e.second;
      eq.op = NUT_P_EQ;
      cs.push_back(PProg{a, c, eq});
    }
    p.where = and_all(cs);
  }
  if (p.preds.size() > NUT_MAX_PRED) return L.fail("more than " + std::to_string(NUT_MAX_PRED) + " WHERE terms");
  if (b.limit) {
    p.has_limit = true;
    p.limit = b.limit->size;
    p.offset = b.limit->offset;
    if (b.limit->with_ties) return L.fail("LIMIT ... WITH TIES is not executed");
  }

  // an aggregate anywhere in a SELECT item (sum(a) / sum(b) too); other functions
  // (abs, toYYYYMMDD, ...) are computed projections of a scan
  std::function<bool(const Expr &)> contains_agg = [&](const Expr &e) {
    if (e.k == EK::FnCall && e.fn() == FnKind::Others && (is_agg_name(e.id.name) || is_distinct_name(e.id.name)))
      return true;
    if (e.k == EK::Subquery) return false;
    for (const Expr &k : e.kids)
      if (contains_agg(k)) return true;
    return false;
  };
  bool has_agg = false;
  for (const QueryExpr &q : b.columns)
    if (contains_agg(q.e)) has_agg = true;
  if (b.group_by || has_agg || b.distinct) {
    // GROUP BY, or aggregates over the whole table (a global aggregate: no keys), or
    // SELECT DISTINCT of 1-2 columns (= GROUP BY those columns, with a hidden COUNT)
    p.kind = NUT_PLAN_GROUPBY;
    if (b.distinct) {
      if (has_agg) return L.fail("DISTINCT over aggregates is not executed");
      for (const QueryExpr &q : b.columns)
        if (!add_key(p, q.e, L)) return false;
      if (p.keys.empty() || p.keys.size() > (size_t)kMaxGroupKeys) return L.fail("SELECT DISTINCT takes 1 to 8 columns");
      if (!p.compiled && p.keys.size() > NUT_MAX_KEYS) return L.fail("DISTINCT over more than 2 columns runs in expression mode");
      PlanAgg cnt{};
      cnt.op = NUT_AGG_COUNT;
      cnt.expr = NUT_EX_COL;
      add_agg(p, cnt);
    }
    if (b.group_by) {
      for (const QueryExpr &k : *b.group_by) {
        // a SELECT alias names its expression (GROUP BY l_year of getYear(d) AS l_year)
        const Expr *ke = &k.e;
        sv name;
        if (column_ref(p, k.e, name) && !k.e.id.qualified)
          for (const QueryExpr &q : b.columns) {
            sv qn;
            if (q.alias && ieq(*q.alias, name) && !(column_ref(p, q.e, qn) && ieq(qn, name))) {
              ke = &q.e;
              break;
            }
          }
        if (!add_key(p, *ke, L)) return false;
      }
      if (p.keys.empty() || p.keys.size() > (size_t)kMaxGroupKeys) return L.fail("GROUP BY takes 1 to 8 keys");
      if (!p.compiled && p.keys.size() > NUT_MAX_KEYS) return L.fail("more than 2 GROUP BY keys run in expression mode");
    }
    for (const QueryExpr &q : b.columns) {
      PlanOut o;
      o.text = expr_text(q.e);
      o.name = q.alias ? std::string(*q.alias) : o.text;
      if (!lower_output(p, q.e, o, L)) return false;
      p.outs.push_back(std::move(o));
    }
    if (b.having) {
      if (!lower_having(p, *b.having, p.having, L)) return false;
      p.has_having = true;
    }
    if (p.aggs.size() > NUT_MAX_AGGS) return L.fail("more than 8 aggregates");
    if (p.vals.size() > NUT_MAX_VALS) return L.fail("aggregates reference more than 4 value columns");
    if (b.order_by) {
      for (const OrderKey &k : *b.order_by) {
        int idx = -1;
        sv name;
        const std::string text = expr_text(k.e.e);
        for (size_t i = 0; i < p.outs.size() && idx < 0; ++i) {
          const PlanOut &o = p.outs[i];
          if (!o.hidden && (ieq(o.name, text) || ieq(o.text, text))) idx = (int)i;
          if (idx < 0 && !o.hidden && column_ref(p, k.e.e, name) && o.kind == OUT_KEY && p.keys[o.a] >= 0 &&
              ieq(p.cols[p.keys[o.a]], name))
            idx = (int)i;
        }
        if (idx < 0 && !having_output(p, k.e.e, idx, L))
          return L.fail("ORDER BY '" + text + "' is neither an output column nor an aggregate");
        p.order.push_back({idx, k.desc});
      }
    }
    if (p.aggs.size() > NUT_MAX_AGGS) return L.fail("more than 8 aggregates (HAVING / ORDER BY included)");
    if (p.vals.size() > NUT_MAX_VALS) return L.fail("aggregates reference more than 4 value columns");
    bool outer = p.join == NUT_JOIN_LEFT || p.join == PJ_FULL;
    for (const nut_plan::JoinStep &js : p.jn)
      outer = outer || js.type == NUT_JOIN_LEFT || js.type == PJ_RIGHT || js.type == PJ_FULL;
    if (!p.compiled && outer)  // NULL-extended rows need aggregate masks
      return L.fail("outer-join aggregates lower to expression mode");
    return true;
  }

  // no GROUP BY, no aggregate: projected columns (several: expression-mode scans only) and
  // computed projections (expression mode: programs evaluated on the selected rows,
  // nut_eval_rows; a CASE branch without ELSE yields NULL)
  sv name;
  if (b.columns.empty()) return L.fail("a plan without GROUP BY projects columns");
  for (const QueryExpr &q : b.columns)
    if (q.e.k == EK::Identifier && q.e.id.wildcard) {
      // SELECT * (the reference's criterion statement `SELECT * FROM table WHERE 1 = 1`):
      // every column the execution binds, in binding order
      if (b.columns.size() != 1 || q.e.id.qualified || q.alias)
        return L.fail("SELECT * is executed alone and unqualified");
      if (!p.compiled) return L.fail("SELECT * runs in expression mode");
      if (p.join >= 0 || !p.jn.empty()) return L.fail("SELECT * over a JOIN is not executed (name the columns)");
      p.star = true;
      std::vector<std::pair<int, bool>> okeys;
      if (b.order_by)
        for (const OrderKey &k : *b.order_by) {
          sv oname;
          if (!column_ref(p, k.e.e, oname)) return L.fail("ORDER BY '" + expr_text(k.e.e) + "' is not a column");
          okeys.push_back({col_index(p, oname), k.desc});
        }
      p.kind = b.order_by ? NUT_PLAN_SORT : NUT_PLAN_FILTER;
      if (b.order_by) {
        p.desc = okeys[0].second;
        p.sort_keys = okeys;
      }
      return true;
    }
  for (size_t j = 0; j < b.columns.size(); ++j) {
    PlanOut o;
    o.kind = OUT_KEY;
    o.a = (int)j;
    if (column_ref(p, b.columns[j].e, name)) {
      p.projs.push_back(col_index(p, name));
      p.proj_val.emplace_back();
      p.proj_mask.emplace_back();
      o.text = std::string(name);
    } else {
      if (!p.compiled) return L.fail("computed projections run in expression mode");
      PProg v, m;
      bool nullable = false;
      if (!lower_nullable(p, b.columns[j].e, v, m, nullable, L)) return false;
      p.projs.push_back(-1);
      p.proj_val.push_back(std::move(v));
      p.proj_mask.push_back(std::move(m));
      o.text = expr_text(b.columns[j].e);
    }
    o.name = b.columns[j].alias ? std::string(*b.columns[j].alias) : o.text;
    p.outs.push_back(o);
  }
  p.proj = p.projs[0];
  // ORDER BY keys: columns of the table, projected or not (an output alias names its column)
  std::vector<std::pair<int, bool>> okeys;
  if (b.order_by) {
    for (const OrderKey &k : *b.order_by) {
      sv oname;
      if (!column_ref(p, k.e.e, oname)) return L.fail("ORDER BY '" + expr_text(k.e.e) + "' is not a column");
      int ci = -1;
      for (size_t j = 0; j < p.outs.size() && ci < 0; ++j)
        if (ieq(oname, p.outs[j].name)) {
          if (p.projs[j] < 0) return L.fail("ORDER BY a computed projection ('" + p.outs[j].name + "') is not executed");
          ci = p.projs[j];
        }
      okeys.push_back({ci >= 0 ? ci : col_index(p, oname), k.desc});
    }
  }
  const bool keys_only = okeys.size() == 1 && p.projs.size() == 1 && okeys[0].first == p.proj;
  if (p.projs.size() > 1 && !p.compiled) return L.fail("a fused scan projects one column");
  if (!okeys.empty() && !keys_only && !p.compiled)
    return L.fail("ORDER BY with other columns than the projected one runs in expression mode");
  // fused scans: one comparison of the projected column (nut_filter_i64); anything else
  // is an expression-mode scan (nut_select_rows, WHERE compiled for the query)
  for (const PlanPred &pr : p.preds) {
    if (pr.col != p.proj) return L.fail("WHERE must test the projected column (single-column scan)");
    if (pr.op >= NUT_IN) return L.fail("IN in a single-column scan");
  }
  if (p.preds.size() > 1) return L.fail("a scan takes one comparison");
  if (b.order_by) {
    p.kind = NUT_PLAN_SORT;
    p.desc = okeys[0].second;
    p.sort_keys = okeys;
  } else {
    p.kind = NUT_PLAN_FILTER;
  }
  return true;
}

// Aggregate queries lower to the precompiled kernel shapes when they fit (column
// comparisons ANDed, the fused expression shapes); anything else — arbitrary
// expressions, OR / NOT / CASE, column-to-column comparisons, more than 6 terms — to
// expression programs compiled for the query (jit.cpp).  Scans stay on the filter kernel.
// USING columns: an unqualified reference binds to the preserved table's column.  FULL
// OUTER preserves both: there an unqualified u means COALESCE(l.u, r.u), which is not
// executed, so it is rejected (qualified l.u / r.u inside aggregates run).
bool resolve_using(nut_plan &p, Lowering &L) {
  for (const auto &u : p.using_cols)
    for (std::string &c : p.cols)
      if (ieq(c, u.first)) {
        if (p.join == PJ_FULL)
          return L.fail("FULL OUTER JOIN ... USING: unqualified '" + u.first +
                        "' (COALESCE of both tables' columns) is not executed; qualify it");
        c = u.second;
      }
  return true;
}

bool lower_query(const Query &q, nut_plan &p, Lowering &L) {
  Lowering L1;
  if (lower_mode(q, p, L1)) return resolve_using(p, L);
  // aggregate plans and scans both retry in expression mode
  nut_plan p2;
  p2.compiled = true;
  Lowering L2;
  if (!lower_mode(q, p2, L2)) return L.fail(L2.err);
  if (!resolve_using(p2, L)) return false;
  p = std::move(p2);
  return true;
}

bool lower(const Statement &st, nut_plan &p, Lowering &L) {
  if (st.k != StmtKind::Select) return L.fail("only SELECT statements execute");
  return lower_query(st.query, p, L);
}

// An uncorrelated scalar subquery in a value position: planned on its own (a global
// aggregate with one output over the same table, no JOIN), executed before the plan; `c`
// becomes a placeholder naming it (resolve_subqueries puts the value in at execution).
bool scalar_subquery(nut_plan &p, const Expr &e, CVal &c, Lowering &L) {
  if (e.k != EK::Subquery || !e.q) return false;
  auto sub = std::make_shared<nut_plan>();
  Lowering Ls;
  if (!lower_query(*e.q, *sub, Ls)) return L.fail("scalar subquery: " + Ls.err);
  int visible = 0;
  for (const PlanOut &o : sub->outs) visible += o.hidden ? 0 : 1;
  if (sub->kind != NUT_PLAN_GROUPBY || !sub->keys.empty() || !sub->key_progs.empty() || visible != 1)
    return L.fail("a scalar subquery executes as a global aggregate with one output (SELECT agg(..) FROM t ..)");
  if (sub->join >= 0 || !sub->subs.empty() || sub->star)
    return L.fail("a scalar subquery executes over one table, without JOIN or nested subqueries");
  if (p.join >= 0) return L.fail("scalar subqueries execute in single-table plans (the query has a JOIN)");
  if (!p.table.empty() && !sub->table.empty() && !ieq(p.table, sub->table))
    return L.fail("scalar subquery over table '" + sub->table + "' (the query reads '" + p.table +
                  "'): subqueries execute over the same table");
  c = CVal{};
  c.is_int = false;
  c.param = (int)p.subs.size();
  p.subs.push_back(std::move(sub));
  return true;
}

// RPN -> infix text, for describe()
std::string prog_text(const nut_plan &p, const PProg &pp) {
  static const char *bin[] = {"", "", "", "+", "-", "*", "/", "%", "div", "<", "<=", ">", ">=", "=", "!=",
                              "and", "or", "xor", "", "&", "|", "^", "", "<<", ">>"};
  std::vector<std::string> st;
  for (const PNode &n : pp) {
    auto pop = [&]() {
      std::string t = st.empty() ? "?" : st.back();
      if (!st.empty()) st.pop_back();
      return t;
    };
    if (n.op == P_LIKE || n.op == P_ILIKE)
      st.push_back("(" + p.cols[n.col] + (n.op == P_LIKE ? " like " : " ilike ") + cval_str(n.c) + ")");
    else if (n.op == NUT_P_COL) st.push_back(p.cols[n.col]);
    else if (n.op == NUT_P_I64 || n.op == NUT_P_F64) st.push_back(cval_str(n.c));
    else if (n.op == NUT_P_DATEPART) {
      static const char *dp[] = {"toYear",      "toMonth",     "toDayOfMonth", "toQuarter",
                                 "toDayOfWeek", "toDayOfYear", "toYYYYMM",     "toYYYYMMDD"};
      st.push_back(std::string(n.arg >= 0 && n.arg < 8 ? dp[n.arg] : "datepart") + "(" + pop() + ")");
    } else if (n.op == NUT_P_NOT || n.op == NUT_P_BITNOT || n.op == NUT_P_ABS || n.op == NUT_P_TO_F64) {
      const char *f = n.op == NUT_P_NOT ? "not" : n.op == NUT_P_BITNOT ? "~" : n.op == NUT_P_ABS ? "abs" : "toFloat64";
      st.push_back(std::string(f) + "(" + pop() + ")");
    } else if (n.op == NUT_P_IF) {
      std::string e = pop(), t = pop(), c = pop();
      st.push_back("if(" + c + ", " + t + ", " + e + ")");
    } else {
      std::string r = pop(), l = pop();
      if (n.op == NUT_P_NE && r == "0" && (l == "1" || l == "0")) st.push_back(l == "1" ? "true" : "false");
      else st.push_back("(" + l + " " + bin[n.op] + " " + r + ")");
    }
  }
  return st.empty() ? "" : st.back();
}

std::string describe(const nut_plan &p) {
  static const char *kinds[] = {"filter", "groupby", "sort"};
  static const char *aggs[] = {"sum", "count", "min", "max"};
  static const char *exprs[] = {"col", "mul", "add", "sub", "mul_1m", "mul_1m_1p"};
  static const int nargs[] = {1, 2, 2, 2, 2, 3};
  std::string o = "{\"kind\":\"";
  o += kinds[p.kind];
  o += "\",\"table\":";
  json_str(o, p.table);
  o += ",\"columns\":[";
  for (size_t i = 0; i < p.cols.size(); ++i) {
    if (i) o += ',';
    json_str(o, p.cols[i]);
  }
  o += "],\"never\":";
  o += p.never ? "true" : "false";
  o += p.compiled ? ",\"mode\":\"compiled\"" : ",\"mode\":\"fused\"";
  if (p.compiled) {
    o += ",\"where_expr\":";
    json_str(o, prog_text(p, p.where));
  }
  o += ",\"where\":[";
  for (size_t i = 0; i < p.preds.size(); ++i) {
    const PlanPred &pr = p.preds[i];
    if (i) o += ',';
    o += "{\"col\":";
    json_str(o, p.cols[pr.col]);
    o += ",\"op\":\"";
    o += kCmpText[pr.op];
    if (pr.op >= NUT_IN) {
      o += "\",\"values\":[";
      for (size_t j = 0; j < pr.set.size(); ++j) o += (j ? ",\"" : "\"") + cval_str(pr.set[j]) + "\"";
      o += "]}";
    } else {
      o += "\",\"value\":\"" + cval_str(pr.c) + "\",\"value_kind\":\"" + (pr.c.is_str ? "string" : pr.c.is_int ? "int" : "decimal") + "\"}";
    }
  }
  o += "]";
  if (p.kind == NUT_PLAN_GROUPBY) {
    o += ",\"keys\":[";
    for (size_t i = 0; i < p.keys.size(); ++i) {
      if (i) o += ',';
      json_str(o, p.keys[i] >= 0 ? p.cols[p.keys[i]] : p.key_text[i]);
    }
    o += "],\"values\":[";
    for (size_t i = 0; i < p.vals.size(); ++i) {
      if (i) o += ',';
      json_str(o, p.cols[p.vals[i]]);
    }
    o += "],\"aggs\":[";
    for (size_t i = 0; i < p.aggs.size(); ++i) {
      const PlanAgg &a = p.aggs[i];
      if (i) o += ',';
      o += "{\"op\":\"";
      o += a.distinct ? "count_distinct" : aggs[a.op];
      o += "\"";
      if (a.distinct) {
        o += ",\"expr\":";
        json_str(o, prog_text(p, a.val));
      }
      if (p.compiled) {
        if (a.op != NUT_AGG_COUNT) {
          o += ",\"expr\":";
          json_str(o, prog_text(p, a.val));
        }
        if (!a.mask.empty()) {
          o += ",\"mask\":";
          json_str(o, prog_text(p, a.mask));
        }
      } else if (a.op != NUT_AGG_COUNT) {
        o += ",\"expr\":\"";
        o += exprs[a.expr];
        o += "\",\"args\":[";
        for (int j = 0; j < nargs[a.expr]; ++j) {
          if (j) o += ',';
          json_str(o, p.cols[p.vals[a.arg[j]]]);
        }
        o += "]";
      }
      o += "}";
    }
    o += "]";
  } else {
    // a computed projection shows as its program (infix)
    auto proj_text = [&](size_t j) {
      return p.projs[j] >= 0 ? p.cols[p.projs[j]] : prog_text(p, p.proj_val[j]);
    };
    o += ",\"column\":";
    json_str(o, p.star ? std::string("*") : proj_text(0));
    if (!p.star && (p.projs.size() > 1 || p.projs[0] < 0)) {
      o += ",\"project\":[";
      for (size_t j = 0; j < p.projs.size(); ++j) {
        if (j) o += ',';
        json_str(o, proj_text(j));
      }
      o += ']';
    }
  }
  if (p.kind == NUT_PLAN_SORT) {
    o += p.desc ? ",\"desc\":true" : ",\"desc\":false";
    o += ",\"sort\":[";
    for (size_t i = 0; i < p.sort_keys.size(); ++i) {
      if (i) o += ',';
      o += "{\"column\":";
      json_str(o, p.cols[p.sort_keys[i].first]);
      o += p.sort_keys[i].second ? ",\"desc\":true}" : ",\"desc\":false}";
    }
    o += ']';
  }
  o += ",\"outputs\":[";
  for (size_t i = 0; i < p.outs.size(); ++i) {
    const PlanOut &u = p.outs[i];
    if (i) o += ',';
    o += "{\"name\":";
    json_str(o, u.name);
    if (u.hidden) o += ",\"hidden\":true";
    o += u.kind == OUT_KEY ? ",\"from\":\"key\",\"index\":" + std::to_string(u.a)
         : u.kind == OUT_AGG ? ",\"from\":\"agg\",\"index\":" + std::to_string(u.a)
         : u.kind == OUT_EXPR ? ",\"from\":\"expr\",\"expr\":" + std::to_string(u.a)
                              : ",\"from\":\"avg\",\"sum\":" + std::to_string(u.a) + ",\"count\":" + std::to_string(u.b);
    o += "}";
  }
  o += "],\"having\":";
  o += p.has_having ? "true" : "false";
  o += ",\"order\":[";
  for (size_t i = 0; i < p.order.size(); ++i) {
    if (i) o += ',';
    o += "{\"output\":" + std::to_string(p.order[i].first) + ",\"desc\":" + (p.order[i].second ? "true" : "false") + "}";
  }
  o += "],\"limit\":";
  o += p.has_limit ? std::to_string(p.limit) : "null";
  if (p.join >= 0) {
    static const char *jn[] = {"inner", "left", "semi", "anti", "full"};
    o += ",\"join\":{\"type\":\"";
    o += jn[p.join];
    o += p.jright ? "\",\"right\":true" : "\",\"right\":false";
    o += ",\"table\":";
    json_str(o, p.jtable);
    o += ",\"aliases\":[";
    json_str(o, p.talias);
    o += ',';
    json_str(o, p.jalias);
    o += ']';
    o += ",\"on\":[";
    json_str(o, p.cols[p.jkey[0]]);
    o += ',';
    json_str(o, p.cols[p.jkey[1]]);
    o += "]}";
    if (!p.jn.empty()) {
      o += ",\"joins\":[";
      for (size_t k = 0; k < p.jn.size(); ++k) {
        if (k) o += ',';
        o += "{\"table\":";
        json_str(o, p.jn[k].table);
        static const char *st[] = {"inner", "left", "semi", "anti", "full", "right"};
        o += ",\"type\":\"";
        o += st[p.jn[k].type];
        o += '"';
        o += ",\"on\":[";
        json_str(o, p.cols[p.jn[k].key[0]]);
        o += ',';
        json_str(o, p.cols[p.jn[k].key[1]]);
        o += "]}";
      }
      o += ']';
    }
  }
  o += ",\"offset\":" + std::to_string(p.offset);
  if (!p.subs.empty()) {  // scalar subqueries, by placeholder index ($subqueryN)
    o += ",\"subqueries\":[";
    for (size_t i = 0; i < p.subs.size(); ++i) o += (i ? "," : "") + describe(*p.subs[i]);
    o += "]";
  }
  o += "}";
  return o;
}

nut_status put_text(const std::string &s, char *buf, size_t cap, size_t *len) {
  if (len) *len = s.size();
  if (buf && cap) {
    size_t n = std::min(cap - 1, s.size());
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  if (cap < s.size() + 1) return fail(NUT_ERR_CAPACITY, "buffer of " + std::to_string(cap) + " bytes < " +
                                                         std::to_string(s.size() + 1) + " needed");
  return NUT_OK;
}

nut_status parse_into(const char *sql, size_t len, nut_stmt *s) {
  size_t bad = 0;
  if (!valid_utf8(sql, len, &bad))
    return fail(NUT_ERR_INVALID_ARG, "sql is not valid UTF-8 (byte " + std::to_string(bad) + ")");
  s->sql.assign(sql, len);
  ParseError pe;
  if (!parse(sv(s->sql), s->st, pe)) return fail(NUT_ERR_PARSE, pe.str());
  return NUT_OK;
}

// ------------------------------------------------------------------ predicate resolution
enum Verdict { V_PRED, V_TRUE, V_FALSE };

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
  return nullptr;
}

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
bool needs_key_progs(const nut_plan &p) {
  if (!p.compiled || p.kind != NUT_PLAN_GROUPBY) return false;
  if (p.keys.size() > NUT_MAX_KEYS) return true;
  for (int k : p.keys)
    if (k < 0) return true;
  for (const PlanAgg &a : p.aggs)
    if (a.distinct) return true;
  return false;
}
nut_status build_spec(const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts, uint64_t n,
                      nut_agg_spec &s, ProgStore &store, std::vector<int> &agg_f64, GbExtra *gx = nullptr);
PProg and_all(const std::vector<PProg> &cs);
PProg pred_prog(const PlanPred &pr);

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
  for (const auto &k : p.sort_keys) {
    if (dicts && dicts[k.first])
      return fail(NUT_ERR_PLAN, "ORDER BY string column '" + p.cols[k.first] + "' is not executed (dictionary codes "
                                "are in first-seen order)");
    if (bound[k.first]->type != NUT_T_I64 && bound[k.first]->type != NUT_T_F64)
      return fail(NUT_ERR_PLAN, "ORDER BY column '" + p.cols[k.first] + "' must be int64 or float64");
  }
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
    if (computed_proj(p, j)) dc = p.proj_val[j].size() == 1 && p.proj_val[j][0].op == NUT_P_COL ? p.proj_val[j][0].col : -1;
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

nut_status exec_scan(nut_ctx *c, const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts,
                     uint64_t n, nut_result *r) {
  bool computed = false;
  for (size_t j = 0; j < p.projs.size(); ++j) computed = computed || computed_proj(p, j);
  if (computed || (p.kind == NUT_PLAN_SORT &&
                   !(p.sort_keys.size() == 1 && p.projs.size() == 1 && p.sort_keys[0].first == p.proj)))
    return exec_sort_rows(c, p, bound, dicts, n, r);
  const nut_column *col = bound[p.proj];
  if (!p.compiled && p.kind == NUT_PLAN_FILTER && dicts && dicts[p.proj]) {
    // a string column: rerun as an expression-mode scan (codes gathered, then decoded)
    nut_plan q = p;
    std::vector<PProg> cs;
    for (const PlanPred &pr : p.preds) cs.push_back(pred_prog(pr));
    q.compiled = true;
    q.preds.clear();
    q.where = and_all(cs);
    return exec_scan(c, q, bound, dicts, n, r);
  }
  // string columns: expression-mode FILTER scans gather their codes and decode on output
  for (int pj : p.projs)
    if (dicts && dicts[pj] && !(p.compiled && p.kind == NUT_PLAN_FILTER))
      return fail(NUT_ERR_PLAN, "column '" + p.cols[pj] + "' holds strings: sorts and single-column fused scans of "
                                "strings are not executed");
  for (const PlanPred &pr : p.preds)
    if (pr.c.is_str) return fail(NUT_ERR_PLAN, "string constant " + cval_str(pr.c) + " compared with an int64 column");
  // fused scans and sorts: int64; expression-mode FILTER scans: int64 or float64 columns
  for (int pj : p.projs)
    if (bound[pj]->type != NUT_T_I64 && !(p.compiled && p.kind == NUT_PLAN_FILTER && bound[pj]->type == NUT_T_F64))
      return fail(NUT_ERR_PLAN, "column '" + p.cols[pj] + "' must be int64 for this scan/sort");
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

// HAVING evaluation for group i: operands are int64 or f64 output words / constants;
// int-int comparisons are exact, anything else compares as f64
struct HVal {
  bool is_int;
  int64_t i;
  double f;
};
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
    if (op == NUT_P_COL) {
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
        if (d->strs.size() > (size_t)INT32_MAX)
          return fail(NUT_ERR_PLAN, "LIKE over a dictionary of more than 2^31 strings");
        table.resize(d->strs.size());
        for (size_t i = 0; i < d->strs.size(); ++i) table[i] = like_match(d->strs[i], n.c.s, ci);
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
        st = resolve(g.val, s.agg_val[k], "aggregate argument", &t);
        agg_f64[a] = t == NUT_PT_F64;
      }
      if (!st && !g.mask.empty()) st = resolve(g.mask, s.agg_mask[k], "aggregate argument", &t);
    }
    for (size_t j = 0; j < p.key_progs.size() && !st && keyprog && gx; ++j) {
      // a plain string column is a key of dictionary codes; computed keys are numbers
      gx->key.emplace_back();
      st = resolve(p.key_progs[j], gx->key.back(), "GROUP BY key", &t, p.keys[j] >= 0);
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

nut_status exec_groupby(nut_ctx *c, const nut_plan &p, const nut_column *const *bound, const Dict *const *dicts,
                        uint64_t n, uint64_t hint, nut_result *r) {
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
      if (dicts && p.keys[o.a] >= 0 && dicts[p.keys[o.a]]) {
        type = NUT_T_STR;
        out_dict[j] = dicts[p.keys[o.a]];
      }
      for (uint64_t i = 0; i < ng; ++i) col[i] = (uint64_t)keys[i * nk + o.a];
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
          double a, b;
          memcpy(&a, &col[x], 8);
          memcpy(&b, &col[y], 8);
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

}  // namespace

// ====================================================================== C ABI
namespace {

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
        if (nd.op == NUT_P_COL || nd.op == P_LIKE || nd.op == P_ILIKE) read.push_back(nd.col);
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
                     const Dict *const *ldict = nullptr, const Dict *const *rdict = nullptr) {
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
      if ((nd.op == NUT_P_COL || nd.op == P_LIKE || nd.op == P_ILIKE) && nd.col == i) return true;
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
        if (nd.op == NUT_P_COL || nd.op == P_LIKE || nd.op == P_ILIKE) sd = sd < 0 || sd == side[nd.col] ? side[nd.col] : 2;
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

}  // namespace

namespace {

// A chain of INNER joins (nut_plan_executen): FROM t0 JOIN t1 ON .. JOIN t2 ON ..  Single-
// table WHERE conjuncts are pushed down per table; the accumulated join result is kept as
// one row-id array per joined table (the probe side); each step builds on the next table.
// tdicts (typed tables, nut_table_executen): per table, the dictionary of each column
// (NULL = numeric); string columns filter, group and project with their own table's codes.
nut_status exec_joinn(nut_ctx *c, const nut_plan &p, const nut_column *const *tabs, const int *ncols,
                      const uint64_t *nrows, int nt, uint64_t hint, nut_result *r,
                      const Dict *const *const *tdicts = nullptr) {
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
  std::vector<int> side(nc);
  std::vector<const nut_column *> src(nc);
  std::vector<const Dict *> sdict(nc + 1, nullptr);
  for (size_t i = 0; i < nc; ++i) {
    const std::string &nm = p.cols[i];
    int hit = -1, nh = 0;
    for (int t = 0; t < nt; ++t)
      if (find(nm, t)) hit = t, ++nh;
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
    if (col->type != NUT_T_I64 && col->type != NUT_T_F64)
      return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: column '" + nm + "' has an unknown type");
    if (nrows[hit] && !col->data) return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: column '" + nm + "' is NULL");
    side[i] = hit;
    src[i] = col;
    if (tdicts && tdicts[hit]) sdict[i] = tdicts[hit][col - tabs[hit]];
  }
  std::vector<int> knew(nt - 1), kold(nt - 1);
  for (int k = 0; k + 1 < nt; ++k) {
    const int a = p.jn[k].key[0], b = p.jn[k].key[1], t = k + 1;
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
      if ((nd.op == NUT_P_COL || nd.op == P_LIKE || nd.op == P_ILIKE) && nd.col == i) return true;
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
        if (nd.op == NUT_P_COL || nd.op == P_LIKE || nd.op == P_ILIKE) sd = sd < 0 || sd == side[nd.col] ? side[nd.col] : nt;
      (sd >= 0 && sd < nt ? push[sd] : keep).push_back(std::move(cj));
    }
    p2.where = and_all(keep);
  } else {
    p2.preds.clear();
    for (const PlanPred &pr : p.preds) push[side[pr.col]].push_back(pred_prog(pr));
  }
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
    for (;;) {
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

// NUT_COL_HOST columns: copied into stream-ordered HBM for one execute call
struct HostStage {
  std::vector<nut_column> cols;
  std::deque<DevBuf> bufs;
};

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

}  // namespace

extern "C" {

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

}  // namespace

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

void nut_plan_free(nut_plan *p) { delete p; }

nut_status nut_plan_execute(nut_ctx *c, const nut_plan *p, const nut_column *cols, int ncols, uint64_t nrows,
                            uint64_t group_hint, nut_result **out) {
  if (!c || !p || !out || (ncols && !cols) || ncols < 0) return fail(NUT_ERR_INVALID_ARG, "nut_plan_execute: NULL argument");
  *out = nullptr;
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
  if (p->join < 0) return nut_plan_execute(c, p, left, nleft, lrows, group_hint, out);
  if (!p->subs.empty()) return fail(NUT_ERR_UNSUPPORTED, "scalar subqueries execute in single-table plans");
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
  if (p->jn.empty()) {
    if (ntables == 1) return nut_plan_execute(c, p, tables[0], ncols[0], nrows[0], group_hint, out);
    if (ntables == 2)
      return nut_plan_execute2(c, p, tables[0], ncols[0], nrows[0], tables[1], ncols[1], nrows[1], group_hint, out);
    return fail(NUT_ERR_INVALID_ARG, "nut_plan_executen: the plan joins fewer tables");
  }
  if (!p->subs.empty()) return fail(NUT_ERR_UNSUPPORTED, "scalar subqueries execute in single-table plans");
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
  for (size_t i = 0; i < p->cols.size(); ++i) {
    const TCol *tc = nullptr;
    for (const TCol &x : t->cols)
      if (ieq(x.name, p->cols[i])) tc = &x;
    if (!tc) return fail(NUT_ERR_PLAN, "table '" + t->name + "' has no column '" + p->cols[i] + "'");
    cols[i] = nut_column{tc->name.c_str(), tc->dev, tc->exec_type};
    bound[i] = &cols[i];
    dicts[i] = tc->dict;
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
  if (p->join < 0) return nut_table_execute(c, left, p, group_hint, out);
  if (!p->subs.empty()) return fail(NUT_ERR_UNSUPPORTED, "scalar subqueries execute in single-table plans");
  *out = nullptr;
  std::vector<nut_column> cols[2];
  std::vector<const Dict *> dicts[2];
  nut_table *t2[2] = {left, right};
  for (int k = 0; k < 2; ++k) {
    nut_table *t = t2[k];
    if (t->ragged()) return fail(NUT_ERR_INVALID_ARG, "nut_table_execute2: table '" + t->name + "' has ragged columns");
    if (t->device >= 0 && t->device != c->device)
      return fail(NUT_ERR_INVALID_ARG, "nut_table_execute2: table '" + t->name + "' lives on another device");
    for (const TCol &x : t->cols) {
      cols[k].push_back(nut_column{x.name.c_str(), x.dev, x.exec_type});
      dicts[k].push_back(x.dict);
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
  if (p->jn.empty()) {
    if (ntables == 1) return nut_table_execute(c, tables[0], p, group_hint, out);
    if (ntables == 2) return nut_table_execute2(c, tables[0], tables[1], p, group_hint, out);
    return fail(NUT_ERR_INVALID_ARG, "nut_table_executen: the plan joins fewer tables");
  }
  if (!p->subs.empty()) return fail(NUT_ERR_UNSUPPORTED, "scalar subqueries execute in single-table plans");
  *out = nullptr;
  std::vector<std::vector<nut_column>> cols(ntables);
  std::vector<std::vector<const Dict *>> dicts(ntables);
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
      dicts[k].push_back(x.dict);
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
