// sql_lower.cpp — plan lowering: the reference's statement tree -> nut_plan.
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
#include <functional>

#include "sql_plan.hpp"

namespace nut {
namespace plan {

// ------------------------------------------------------------------ plan
const char *kCmpText[] = {"<", "<=", ">", ">=", "=", "!=", "in", "not in"};


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



int pnode_arity(int op) {
  if (op == P_LIKE || op == P_ILIKE || op == P_SUBSTR) return 0;
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
// Inside an EXISTS / IN subquery (p.scope >= 1) an unqualified name is scoped: it binds to
// the subquery's table first, then to the outer query's (a correlation).
bool column_ref(nut_plan &p, const Expr &e, sv &name) {
  if (e.k != EK::Identifier || e.id.wildcard) return false;
  if (e.id.qualified && (p.join >= 0 || !(ieq(e.id.qualifier, p.table) || (!p.talias.empty() && ieq(e.id.qualifier, p.talias))))) {
    // a JOIN plan's qualified name, or a single-table plan's with another qualifier
    // (n1.n_name of a flat table: bound to a column of that name, else to n_name)
    p.qnames.push_back(std::string(e.id.qualifier) + "." + std::string(e.id.name));
    name = p.qnames.back();
  } else if (p.scope > 0) {
    p.qnames.push_back(scoped_name(p.scope, e.id.name));
    name = p.qnames.back();
  } else {
    name = e.id.name;
  }
  return true;
}

std::string scoped_name(int scope, sv name) {
  return "\x1f" + std::to_string(scope) + "\x1f" + std::string(name);
}

int name_scope(const std::string &name, std::string *bare) {
  if (name.size() < 3 || name[0] != '\x1f') {
    if (bare) *bare = name;
    return 0;
  }
  const size_t e = name.find('\x1f', 1);
  if (e == std::string::npos) {
    if (bare) *bare = name;
    return 0;
  }
  if (bare) *bare = name.substr(e + 1);
  return atoi(name.c_str() + 1);
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
  if (a.size() == 1 && a[0].op == NUT_P_I64 && a[0].c.is_str && other.size() == 1 &&
      (other[0].op == NUT_P_COL || other[0].op == P_SUBSTR))  // (substrings: codes of the column's dictionary)
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
      if ((ieq(n, "substring") || ieq(n, "substr") || ieq(n, "mid")) && (na == 2 || na == 3)) {
        // substring(col, offset[, length]) of a string column, constant offset / length:
        // a dictionary function (P_SUBSTR: the codes map to the substrings' codes)
        sv cname;
        CVal off, len;
        len.v = kHuge;
        if (!column_ref(p, e.kids[0], cname) || !const_eval(e.kids[1], off, L) || !off.is_int || off.is_str ||
            off.param >= 0 || (na == 3 && (!const_eval(e.kids[2], len, L) || !len.is_int || len.is_str || len.param >= 0)))
          return L.fail("substring takes a string column and integer constants ('" + expr_text(e) + "')");
        if (off.v < INT32_MIN || off.v > INT32_MAX) return L.fail("substring offset out of range ('" + expr_text(e) + "')");
        PNode sn;
        sn.op = P_SUBSTR;
        sn.col = col_index(p, cname);
        sn.arg = (int)off.v;
        sn.c = len;
        o.push_back(sn);
        return true;
      }
      if (ieq(n, "todate")) return L.fail("toDate takes one 'YYYY-MM-DD' constant");
      return L.fail("function '" + std::string(n) + "' is not executed (executed: if, multiIf, abs, toFloat64, intDiv, "
                    "modulo, substring, toYear/getYear, toMonth, toDayOfMonth, toQuarter, toDayOfWeek, toDayOfYear, toYYYYMM, "
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
        if (reads_col(nd.op)) a.refs.push_back(nd.col);
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
        if (reads_col(nd.op)) a.refs.push_back(nd.col);
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
// ON split into its column = column equalities (the keys) and its other conjuncts (`rest`:
// filters of the JOIN source's table)
void on_split(nut_plan &p, const Expr &e, std::vector<std::pair<int, int>> &eqs, std::vector<const Expr *> &rest) {
  if (e.k == EK::BinaryOp && e.bop() == BinOp::And) {
    on_split(p, e.kids[0], eqs, rest);
    on_split(p, e.kids[1], eqs, rest);
    return;
  }
  sv ka, kb;
  if (e.k == EK::BinaryOp && e.bop() == BinOp::Eq && column_ref(p, e.kids[0], ka) && column_ref(p, e.kids[1], kb)) {
    const int a = col_index(p, ka);
    eqs.emplace_back(a, col_index(p, kb));
  } else {
    rest.push_back(&e);
  }
}

// the ON filters as one program (expression mode): and_all of each conjunct's
bool on_filters(nut_plan &p, const std::vector<const Expr *> &rest, PProg &cond, Lowering &L) {
  if (rest.empty()) return true;
  if (!p.compiled) return L.fail("JOIN ON conditions beyond key equalities run in expression mode");
  std::vector<PProg> cs;
  for (const Expr *e : rest) {
    PProg c;
    if (!lower_prog(p, *e, c, L)) return false;
    cs.push_back(std::move(c));
  }
  cond = and_all(cs);
  return true;
}

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

// ---- EXISTS / NOT EXISTS (subquery), x [NOT] IN (subquery) as SEMI / ANTI join steps
// (DESIGN.md §3.8).  The reference parses them (TPC-H Q4 / Q16 / Q21 = its fixtures
// tests/sql/2.sql:9-17, 7.sql:13-20, 8.sql:11-27); this executes the correlated shapes: the
// subquery reads one table, its WHERE is an AND chain holding one equality with the outer
// query (EXISTS; for IN, the projected column = x is the key), filters of its own table,
// and at most one other comparison between its table and the outer query.

// the AND chain's conjuncts, in order
void and_conjuncts(const Expr &e, std::vector<const Expr *> &out) {
  if (e.k == EK::BinaryOp && e.bop() == BinOp::And) {
    and_conjuncts(e.kids[0], out);
    and_conjuncts(e.kids[1], out);
  } else {
    out.push_back(&e);
  }
}

// e is `[NOT] EXISTS (subquery)` or `x [NOT] IN (subquery)`: *sq = the subquery expression,
// *x = the IN operand (NULL for EXISTS), *neg = NOT EXISTS / NOT IN
bool semi_conjunct(const Expr &e, const Expr **sq, const Expr **x, bool *neg) {
  bool n = false;
  const Expr *f = &e;
  if (f->k == EK::UnaryOp && f->uop() == UnOp::Not) {  // prefix NOT binds to exists(...)
    n = true;
    f = &f->kids[0];
  }
  if (f->k == EK::FnCall && f->kids.size() == 1 && f->kids[0].k == EK::Subquery &&
      (f->fn() == FnKind::Exists || f->fn() == FnKind::NotExists || (f->fn() == FnKind::Others && ieq(f->id.name, "exists")))) {
    *sq = &f->kids[0];
    *x = nullptr;
    *neg = n != (f->fn() == FnKind::NotExists);
    return true;
  }
  if (!n && f->k == EK::BinaryOp && (f->bop() == BinOp::In || f->bop() == BinOp::NotIn) && f->kids[1].k == EK::Subquery) {
    *sq = &f->kids[1];
    *x = &f->kids[0];
    *neg = f->bop() == BinOp::NotIn;
    return true;
  }
  return false;
}

bool lower_semi(nut_plan &p, const Expr &sq, const Expr *x, bool neg, Lowering &L) {
  const char *what = x ? (neg ? "NOT IN (subquery)" : "IN (subquery)") : (neg ? "NOT EXISTS" : "EXISTS");
  auto bad = [&](const std::string &m) { return L.fail(std::string(what) + ": " + m); };
  if (!sq.q || sq.q->is_union) return bad("UNION subqueries are not executed");
  const QueryBody &b = *sq.q->body;
  if (b.with || b.distinct || b.group_by || b.having || b.order_by || b.limit)
    return bad("the subquery may have WHERE only (no WITH / DISTINCT / GROUP BY / HAVING / ORDER BY / LIMIT)");
  if (!b.from || b.from->k != SourceKind::Table) return bad("the subquery must read one table");
  if (!b.joins.empty()) return bad("a subquery with JOIN is not executed");
  for (const QueryExpr &c : b.columns)
    if (c.e.k == EK::FnCall && c.e.fn() == FnKind::Others && is_agg_name(c.e.id.name))
      return bad("an aggregate subquery is not a row set");
  nut_plan::JoinStep js;
  js.type = neg ? NUT_JOIN_ANTI : NUT_JOIN_SEMI;
  js.table = std::string(b.from->table);
  if (b.from->alias) js.alias = std::string(*b.from->alias);
  int nscope = 1;
  for (const nut_plan::JoinStep &o : p.jn) nscope = std::max(nscope, o.scope + 1);
  js.scope = nscope;
  sv name;
  if (x) {  // x [NOT] IN (SELECT y FROM t ...): the key pair (x, y)
    if (b.columns.size() != 1) return bad("the subquery must select one column");
    if (!column_ref(p, *x, name)) return bad("the IN operand must be a column");
    js.key[0] = col_index(p, name);
    p.scope = js.scope;
    const bool ok = column_ref(p, b.columns[0].e, name);
    p.scope = 0;
    if (!ok) return bad("the subquery must select a column");
    js.key[1] = col_index(p, name);
  }
  if (b.where) {
    bool wb;
    p.scope = js.scope;
    const size_t nsubs = p.subs.size();
    bool ok = true;
    if (b.where->is_bool_lit(&wb)) {
      if (!wb) {
        PNode f;
        f.op = NUT_P_I64;
        f.c.v = 0;
        js.cond.push_back(f);
      }
    } else {
      ok = lower_prog(p, *b.where, js.cond, L);
    }
    p.scope = 0;
    if (!ok) return false;
    if (p.subs.size() != nsubs) return bad("a scalar subquery inside it is not executed");
  } else if (!x) {
    return bad("an uncorrelated EXISTS (no WHERE) is not executed");
  }
  p.jn.push_back(std::move(js));
  return true;
}

bool lower_mode(const Query &qry, nut_plan &p, Lowering &L) {
  if (qry.is_union) return L.fail("UNION/INTERSECT/EXCEPT are not executed (one query body per plan)");
  const QueryBody &b = *qry.body;
  if (b.with) return L.fail("WITH is not executed");
  if (b.distinct && b.group_by) return L.fail("DISTINCT with GROUP BY is not executed");
  if (!b.from || b.from->k != SourceKind::Table) return L.fail("FROM must name one table");
  p.table = std::string(b.from->table);
  if (b.from->alias) p.talias = std::string(*b.from->alias);
  // EXISTS / IN subqueries among the WHERE conjuncts: SEMI / ANTI steps of a join chain
  std::vector<const Expr *> wconj;
  bool has_semi = false;
  if (b.where) {
    and_conjuncts(*b.where, wconj);
    for (const Expr *e : wconj) {
      const Expr *sq, *x;
      bool neg;
      has_semi = has_semi || semi_conjunct(*e, &sq, &x, &neg);
    }
  }
  if (has_semi) {
    if (!p.compiled) return L.fail("EXISTS / IN (subquery) run in expression mode");
    if (b.from->alias) p.talias = std::string(*b.from->alias);
    p.join = NUT_JOIN_INNER;  // a chain (qualified names keep their qualifier from here on)
  }
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
      std::vector<const Expr *> rest;
      on_split(p, jc.cond, eqs, rest);
      if (eqs.empty()) return L.fail("JOIN ON needs an equality of two columns (the key)");
      if (eqs.size() > 1 && jc.t != JoinType::Inner)
        return L.fail("JOIN with several key columns: INNER only (outer / semi / anti joins take one ON equality)");
      if (!rest.empty() && (type == PJ_RIGHT || type == PJ_FULL))
        return L.fail("JOIN ON conditions beyond key equalities: INNER, LEFT, SEMI and ANTI joins (they filter the JOIN source)");
      nut_plan::JoinStep js;
      js.type = type;
      if (!on_filters(p, rest, js.cond, L)) return false;
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
    PProg on_cond;                         // ON filters of the JOIN source: the join runs as a one-step chain
    if (jc.on) {
      std::vector<const Expr *> rest;
      on_split(p, jc.cond, eqs, rest);
      if (eqs.empty()) return L.fail("JOIN ON needs an equality of two columns (the key)");
      if (!rest.empty() && (p.jright || p.join == PJ_FULL))
        return L.fail("JOIN ON conditions beyond key equalities: INNER, LEFT, SEMI and ANTI joins (they filter the JOIN source)");
      if (!on_filters(p, rest, on_cond, L)) return false;
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
    if (has_semi || !on_cond.empty()) {  // the one JOIN becomes the first step of a chain (the subqueries extend it)
      if (p.jright && p.join != NUT_JOIN_LEFT) return L.fail("RIGHT SEMI / ANTI JOIN with EXISTS / IN subqueries is not executed");
      if (!p.using_cols.empty()) return L.fail("JOIN ... USING with EXISTS / IN subqueries is not executed (ON a = b)");
      nut_plan::JoinStep js;
      js.table = p.jtable;
      js.alias = p.jalias;
      js.key[0] = p.jkey[0];
      js.key[1] = p.jkey[1];
      js.type = p.jright ? PJ_RIGHT : p.join;
      js.cond = std::move(on_cond);
      p.jn.push_back(js);
      p.join = NUT_JOIN_INNER;
      p.jright = false;
    }
  }
  if (b.having && !b.group_by) return L.fail("HAVING needs GROUP BY");
  p.table = std::string(b.from->table);
  bool wb;
  if (has_semi) {  // the other conjuncts form the WHERE (expression mode)
    std::vector<PProg> cs;
    for (const Expr *e : wconj) {
      const Expr *sq, *x;
      bool neg;
      if (semi_conjunct(*e, &sq, &x, &neg)) {
        if (!lower_semi(p, *sq, x, neg, L)) return false;
        continue;
      }
      if (e->is_bool_lit(&wb)) {
        if (!wb) p.never = true;
        continue;
      }
      PProg c;
      if (!lower_prog(p, *e, c, L)) return false;
      cs.push_back(std::move(c));
    }
    p.where = and_all(cs);
    if (p.jn.size() > 15) return L.fail("at most 16 joined tables (JOINs and EXISTS / IN subqueries)");
    p.jtable = p.jn[0].table;
    p.jalias = p.jn[0].alias;
    p.jkey[0] = p.jn[0].key[0];
    p.jkey[1] = p.jn[0].key[1];
  } else if (p.compiled && b.where) {
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

// ---- derived tables: FROM (SELECT e1 AS a1, ... FROM t [JOIN ..] WHERE w) AS d
// with a projection-only body (no aggregate, GROUP BY, DISTINCT, ORDER BY or LIMIT) is
// flattened into the outer query — the shape of the reference's fixture tests/sql/3.sql
// (TPC-H Q7's `shipping`): every outer reference to a_i (or d.a_i) becomes e_i, the body's
// FROM / JOINs become the outer FROM / JOINs and its WHERE is ANDed to the outer WHERE.
Expr clone_expr(const Expr &e);
std::unique_ptr<Query> clone_query(const Query &q);

QuerySource clone_source(const QuerySource &s) {
  QuerySource o;
  o.k = s.k;
  o.table = s.table;
  o.e = clone_expr(s.e);
  o.alias = s.alias;
  return o;
}

QueryExpr clone_qexpr(const QueryExpr &q) {
  QueryExpr o;
  o.e = clone_expr(q.e);
  o.alias = q.alias;
  return o;
}

std::unique_ptr<Query> clone_query(const Query &q) {
  auto o = std::make_unique<Query>();
  o->is_union = q.is_union;
  o->ut = q.ut;
  if (q.l) o->l = clone_query(*q.l);
  if (q.r) o->r = clone_query(*q.r);
  if (!q.body) return o;
  const QueryBody &b = *q.body;
  o->body = std::make_unique<QueryBody>();
  QueryBody &n = *o->body;
  if (b.with) {
    n.with.emplace();
    for (const CTE &c : *b.with) {
      CTE x;
      x.q = c.q ? clone_query(*c.q) : nullptr;
      x.alias = c.alias;
      n.with->push_back(std::move(x));
    }
  }
  n.distinct = b.distinct;
  if (b.distinct_on) {
    n.distinct_on.emplace();
    for (const QueryExpr &x : *b.distinct_on) n.distinct_on->push_back(clone_qexpr(x));
  }
  for (const QueryExpr &x : b.columns) n.columns.push_back(clone_qexpr(x));
  if (b.from) n.from = clone_source(*b.from);
  for (const JoinClause &j : b.joins) {
    JoinClause x;
    x.t = j.t;
    x.src = clone_source(j.src);
    x.on = j.on;
    x.cond = clone_expr(j.cond);
    x.using_ = j.using_;
    n.joins.push_back(std::move(x));
  }
  if (b.where) n.where = clone_expr(*b.where);
  if (b.group_by) {
    n.group_by.emplace();
    for (const QueryExpr &x : *b.group_by) n.group_by->push_back(clone_qexpr(x));
  }
  if (b.having) n.having = clone_expr(*b.having);
  if (b.order_by) {
    n.order_by.emplace();
    for (const OrderKey &k : *b.order_by) {
      OrderKey x;
      x.e = clone_qexpr(k.e);
      x.desc = k.desc;
      n.order_by->push_back(std::move(x));
    }
  }
  n.limit = b.limit;
  return o;
}

Expr clone_expr(const Expr &e) {
  Expr o;
  o.k = e.k;
  o.op = e.op;
  o.id = e.id;
  o.param = e.param;
  if (e.lit) o.lit = std::make_unique<Literal>(*e.lit);
  for (const Expr &k : e.kids) o.kids.push_back(clone_expr(k));
  if (e.q) o.q = clone_query(*e.q);
  return o;
}

// e with every reference to a derived table's output (unqualified, or qualified by its
// alias d) replaced by the output's expression; subqueries are copied unchanged
Expr subst_derived(const Expr &e, const std::vector<std::pair<sv, const Expr *>> &outs, std::optional<sv> d) {
  if (e.k == EK::Identifier && !e.id.wildcard && (!e.id.qualified || (d && ieq(e.id.qualifier, *d))))
    for (const auto &o : outs)
      if (ieq(o.first, e.id.name)) return clone_expr(*o.second);
  if (e.k == EK::Subquery) return clone_expr(e);
  Expr o;
  o.k = e.k;
  o.op = e.op;
  o.id = e.id;
  o.param = e.param;
  if (e.lit) o.lit = std::make_unique<Literal>(*e.lit);
  for (const Expr &k : e.kids) o.kids.push_back(subst_derived(k, outs, d));
  return o;
}

bool flatten_derived(const Query &q, std::unique_ptr<Query> &flat, Lowering &L) {
  const QueryBody &b = *q.body;
  const QuerySource &src = *b.from;
  if (!src.e.q || src.e.q->is_union || !src.e.q->body) return L.fail("derived table: UNION bodies are not executed");
  const QueryBody &in = *src.e.q->body;
  if (in.with || in.distinct || in.distinct_on || in.group_by || in.having || in.order_by || in.limit)
    return L.fail("derived table: only projection bodies (SELECT exprs FROM .. WHERE ..) are flattened");
  if (!in.from) return L.fail("derived table: its body needs FROM");
  if (!b.joins.empty() && !in.joins.empty()) return L.fail("derived table with JOINs inside a query with JOINs is not executed");
  // the body's outputs by name: its alias, or a column's own name
  std::vector<std::pair<sv, const Expr *>> outs;
  std::function<bool(const Expr &)> has_agg = [&](const Expr &e) {
    if (e.k == EK::FnCall && e.fn() == FnKind::Others && is_agg_name(e.id.name)) return true;
    for (const Expr &k : e.kids)
      if (has_agg(k)) return true;
    return false;
  };
  for (const QueryExpr &c : in.columns) {
    if (c.e.k == EK::Identifier && c.e.id.wildcard) return L.fail("derived table: SELECT * inside it is not executed");
    if (has_agg(c.e)) return L.fail("derived table: aggregates inside it are not executed");
    if (c.alias)
      outs.push_back({*c.alias, &c.e});
    else if (c.e.k == EK::Identifier)
      outs.push_back({c.e.id.name, &c.e});
    else
      return L.fail("derived table: output '" + expr_text(c.e) + "' needs an alias");
  }
  flat = std::make_unique<Query>();
  flat->body = std::make_unique<QueryBody>();
  QueryBody &n = *flat->body;
  const std::optional<sv> d = src.alias;
  n.distinct = b.distinct;
  for (const QueryExpr &c : b.columns) {
    if (c.e.k == EK::Identifier && c.e.id.wildcard) return L.fail("derived table: SELECT * over it is not executed");
    QueryExpr x;
    x.e = subst_derived(c.e, outs, d);
    // a bare reference keeps its name as the output's (ORDER BY / result columns use it)
    x.alias = c.alias ? c.alias : (c.e.k == EK::Identifier ? std::optional<sv>(c.e.id.name) : std::nullopt);
    n.columns.push_back(std::move(x));
  }
  n.from = clone_source(*in.from);
  for (const JoinClause &j : in.joins.empty() ? b.joins : in.joins) {
    JoinClause x;
    x.t = j.t;
    x.src = clone_source(j.src);
    x.on = j.on;
    x.cond = in.joins.empty() ? subst_derived(j.cond, outs, d) : clone_expr(j.cond);
    x.using_ = j.using_;
    n.joins.push_back(std::move(x));
  }
  if (in.where && b.where) {
    Expr a;
    a.k = EK::BinaryOp;
    a.op = (uint8_t)BinOp::And;
    a.kids.push_back(clone_expr(*in.where));
    a.kids.push_back(subst_derived(*b.where, outs, d));
    n.where = std::move(a);
  } else if (in.where) {
    n.where = clone_expr(*in.where);
  } else if (b.where) {
    n.where = subst_derived(*b.where, outs, d);
  }
  if (b.group_by) {
    n.group_by.emplace();
    for (const QueryExpr &k : *b.group_by) {
      QueryExpr x;
      x.e = subst_derived(k.e, outs, d);
      x.alias = k.alias;
      n.group_by->push_back(std::move(x));
    }
  }
  if (b.having) n.having = subst_derived(*b.having, outs, d);
  if (b.order_by) {
    n.order_by.emplace();
    for (const OrderKey &k : *b.order_by) {
      OrderKey x;
      // an output alias of the outer SELECT stays a name (it is matched to an output)
      bool outer_alias = false;
      if (k.e.e.k == EK::Identifier && !k.e.e.id.qualified)
        for (const QueryExpr &c : b.columns)
          outer_alias = outer_alias || (c.alias && ieq(*c.alias, k.e.e.id.name));
      x.e.e = outer_alias ? clone_expr(k.e.e) : subst_derived(k.e.e, outs, d);
      x.e.alias = k.e.alias;
      x.desc = k.desc;
      n.order_by->push_back(std::move(x));
    }
  }
  n.limit = b.limit;
  return true;
}

// a derived table whose body groups or aggregates: materialized (nut_plan::inner) when the
// outer query reads it alone (no JOIN), by name, as its own table
bool grouped_body(const QueryBody &in) {
  std::function<bool(const Expr &)> has_agg = [&](const Expr &e) {
    if (e.k == EK::FnCall && e.fn() == FnKind::Others && is_agg_name(e.id.name)) return true;
    for (const Expr &k : e.kids)
      if (has_agg(k)) return true;
    return false;
  };
  if (in.group_by) return true;
  for (const QueryExpr &c : in.columns)
    if (has_agg(c.e)) return true;
  return false;
}

// the number of columns a plan outputs (-1: SELECT *, known at execution)
int visible_columns(const nut_plan &p) {
  if (p.kind != NUT_PLAN_GROUPBY) return p.star ? -1 : (int)p.projs.size();
  int n = 0;
  for (const PlanOut &o : p.outs) n += o.hidden ? 0 : 1;
  return n;
}

bool lower_query(const Query &q, nut_plan &p, Lowering &L) {
  if (q.is_union) {  // UNION ALL: every branch its own plan, the results concatenated (§3.9)
    std::vector<const Query *> br;
    std::function<bool(const Query &)> collect = [&](const Query &x) -> bool {
      if (!x.is_union) {
        br.push_back(&x);
        return true;
      }
      return x.ut == UnionType::UnionAll && x.l && x.r && collect(*x.l) && collect(*x.r);
    };
    if (!collect(q)) return L.fail("UNION [DISTINCT], INTERSECT and EXCEPT are not executed (UNION ALL is)");
    for (size_t k = 0; k < br.size(); ++k) {
      auto bp = std::make_shared<nut_plan>();
      Lowering Lb;
      const std::string which = "UNION ALL branch " + std::to_string(k + 1) + ": ";
      if (!lower_query(*br[k], *bp, Lb)) return L.fail(which + Lb.err);
      if (bp->join >= 0 || !bp->jn.empty() || bp->inner || !bp->uni.empty())
        return L.fail(which + "a branch executes over one table (no JOIN or derived table)");
      if (k && (bp->kind == NUT_PLAN_GROUPBY) != (p.uni[0]->kind == NUT_PLAN_GROUPBY))
        return L.fail("UNION ALL: every branch a scan, or every branch an aggregate");
      if (k && visible_columns(*bp) >= 0 && visible_columns(*p.uni[0]) >= 0 &&
          visible_columns(*bp) != visible_columns(*p.uni[0]))
        return L.fail("UNION ALL: the branches output different numbers of columns");
      p.uni.push_back(bp);
    }
    p.kind = p.uni[0]->kind;
    p.table = p.uni[0]->table;
    for (const auto &b : p.uni)
      for (const std::string &c : b->cols)
        if (std::find(p.cols.begin(), p.cols.end(), c) == p.cols.end()) p.cols.push_back(c);
    return true;
  }
  // WITH name AS (query) ... FROM name [alias]: the CTE as a derived table
  if (!q.is_union && q.body && q.body->with && q.body->from && q.body->from->k == SourceKind::Table) {
    const QuerySource &f = *q.body->from;
    for (const CTE &c : *q.body->with) {
      if (!c.q || !ieq(c.alias, f.table)) continue;
      auto n = clone_query(q);
      n->body->with.reset();
      QuerySource d;
      d.k = SourceKind::Subquery;
      d.e.k = EK::Subquery;
      d.e.q = clone_query(*c.q);
      d.alias = f.alias ? f.alias : std::optional<sv>(c.alias);
      n->body->from = std::move(d);
      return lower_query(*n, p, L);
    }
    return L.fail("WITH: the query reads no CTE from FROM (CTEs in JOINs or subqueries are not executed)");
  }
  if (!q.is_union && q.body && q.body->with) return L.fail("WITH: a CTE is executed when FROM names it");
  if (!q.is_union && q.body && q.body->from && q.body->from->k == SourceKind::Subquery) {
    const QuerySource &src = *q.body->from;
    const bool grouped = src.e.q && !src.e.q->is_union && src.e.q->body && grouped_body(*src.e.q->body);
    if (grouped) {
      if (!q.body->joins.empty()) return L.fail("derived table: a grouped derived table is not joined");
      auto inner = std::make_shared<nut_plan>();
      Lowering Li;
      if (!lower_query(*src.e.q, *inner, Li)) return L.fail("derived table: " + Li.err);
      if (inner->kind != NUT_PLAN_GROUPBY) return L.fail("derived table: its grouped body must lower to a group-by");
      for (const PlanOut &o : inner->outs)
        if (o.name.empty() && !o.hidden) return L.fail("derived table: every output of its body needs a name");
      // the outer query over a table named by the derived table's alias
      auto n = clone_query(q);
      QuerySource t;
      t.k = SourceKind::Table;
      t.table = src.alias ? *src.alias : sv("derived");
      n->body->from = std::move(t);
      if (!lower_query(*n, p, L)) return false;
      if (p.join >= 0 || !p.jn.empty()) return L.fail("derived table: a grouped derived table is not joined");
      p.inner = std::move(inner);
      return true;
    }
    std::unique_ptr<Query> flat;
    if (!flatten_derived(q, flat, L)) return false;
    return lower_query(*flat, p, L);
  }
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
  // CREATE VIEW v AS query: the rows the view holds — its query (the reference's fixture
  // tests/sql/12.sql, a UNION ALL of four tables); nothing is stored
  if (st.k == StmtKind::Create && st.is_view && st.view) return lower_query(st.view->query, p, L);
  if (st.k != StmtKind::Select) return L.fail("only SELECT statements (and CREATE VIEW bodies) execute");
  return lower_query(st.query, p, L);
}

// An uncorrelated scalar subquery in a value position: planned on its own (a global
// aggregate with one output over the plan's FROM table, no JOIN — in a JOIN plan too:
// table 0 of the execution), executed before the plan; `c`
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
  if (!p.table.empty() && !sub->table.empty() && !ieq(p.table, sub->table))
    return L.fail("scalar subquery over table '" + sub->table + "' (the query reads '" + p.table +
                  "'): subqueries execute over the same table");
  c = CVal{};
  c.is_int = false;
  c.param = (int)p.subs.size();
  p.subs.push_back(std::move(sub));
  return true;
}

// a plan column's name as describe() shows it (subquery scope n: "sub<n>:name")
std::string shown(const std::string &name) {
  std::string bare;
  const int sc = name_scope(name, &bare);
  return sc ? "sub" + std::to_string(sc) + ":" + bare : name;
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
      st.push_back("(" + shown(p.cols[n.col]) + (n.op == P_LIKE ? " like " : " ilike ") + cval_str(n.c) + ")");
    else if (n.op == P_SUBSTR)
      st.push_back("substring(" + shown(p.cols[n.col]) + ", " + std::to_string(n.arg) +
                   (n.c.v >= kHuge ? std::string() : ", " + i128_str(n.c.v)) + ")");
    else if (n.op == NUT_P_COL) st.push_back(shown(p.cols[n.col]));
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
  // (a materialized derived table: the columns the caller binds are its body's; this
  // plan's own, over the body's outputs, are "derived_columns")
  const std::vector<std::string> &bcols = p.inner ? p.inner->cols : p.cols;
  o += ",\"columns\":[";
  for (size_t i = 0; i < bcols.size(); ++i) {
    if (i) o += ',';
    json_str(o, shown(bcols[i]));
  }
  if (p.inner) {
    o += "],\"derived_columns\":[";
    for (size_t i = 0; i < p.cols.size(); ++i) {
      if (i) o += ',';
      json_str(o, shown(p.cols[i]));
    }
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
    json_str(o, p.star ? std::string("*") : p.projs.empty() ? std::string() : proj_text(0));  // (UNION ALL: its branches)
    if (!p.star && (p.projs.size() > 1 || (!p.projs.empty() && p.projs[0] < 0))) {
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
    o += ",\"on\":";
    if (p.jkey[0] >= 0) {
      o += '[';
      json_str(o, shown(p.cols[p.jkey[0]]));
      o += ',';
      json_str(o, shown(p.cols[p.jkey[1]]));
      o += ']';
    } else {
      o += "null";
    }
    o += '}';
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
        o += ",\"on\":";
        if (p.jn[k].key[0] >= 0) {
          o += '[';
          json_str(o, shown(p.cols[p.jn[k].key[0]]));
          o += ',';
          json_str(o, shown(p.cols[p.jn[k].key[1]]));
          o += ']';
        } else {
          o += "null";
        }
        if (p.jn[k].scope) {
          o += ",\"subquery\":" + std::to_string(p.jn[k].scope) + ",\"alias\":";
          json_str(o, p.jn[k].alias);
          o += ",\"where\":";
          json_str(o, prog_text(p, p.jn[k].cond));
        } else if (!p.jn[k].cond.empty()) {  // ON filters of the step's table
          o += ",\"on_filter\":";
          json_str(o, prog_text(p, p.jn[k].cond));
        }
        o += '}';
      }
      o += ']';
    }
  }
  o += ",\"offset\":" + std::to_string(p.offset);
  if (p.inner) o += ",\"derived\":" + describe(*p.inner);
  if (!p.uni.empty()) {  // UNION ALL: the branches, in order
    o += ",\"union_all\":[";
    for (size_t i = 0; i < p.uni.size(); ++i) o += (i ? "," : "") + describe(*p.uni[i]);
    o += "]";
  }
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


}  // namespace plan
}  // namespace nut
