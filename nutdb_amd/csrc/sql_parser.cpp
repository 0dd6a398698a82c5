// sql_parser.cpp — top-down operator-precedence parser of the NutDB SQL dialect.
//
// C++ restatement of /root/reference/src/parser/mod.rs (Parser, 1974 lines), with
// literal decoding from literal.rs and constant folding from simplify.rs.  Accepts and
// rejects exactly what the reference does, including its quirks:
//   - ORDER BY tests DESC twice and never consumes ASC (mod.rs:491-495), so
//     "ORDER BY k ASC" fails with "more than one statement";
//   - a $n parameter demands a further integer literal (mod.rs:1311);
//   - prefix NOT binds to the next prefix only (mod.rs:1294-1296);
//   - Map(K, V) is stored as (V, K) (mod.rs:1780);
//   - only the first statement is checked: text after ';' is never tokenized
//     (mod.rs:164-167).
// Errors carry the reference's Display text (error.rs:8-57, tokenizer/error.rs).
#include <stdlib.h>
#include <string.h>

#include <initializer_list>

#include "sql_ast.hpp"
#include "sql_lexer.hpp"

namespace nut::sql {

// ============================================================== AST plumbing
Expr::Expr() = default;
Expr::Expr(Expr &&) noexcept = default;
Expr &Expr::operator=(Expr &&) noexcept = default;
Expr::~Expr() = default;

static std::string strip_zeros(const std::string &d) {
  size_t i = 0;
  while (i < d.size() && d[i] == '0') ++i;
  return d.substr(i);
}

bool Decimal::operator==(const Decimal &o) const {
  // BigDecimal PartialEq (bigdecimal 0.3): compare after aligning scales
  if (is_zero() || o.is_zero()) return is_zero() && o.is_zero();
  if (neg != o.neg) return false;
  auto norm = [](const Decimal &d, std::string &dig, int64_t &sc) {
    dig = d.digits;
    sc = d.scale;
    while (!dig.empty() && dig.back() == '0') {
      dig.pop_back();
      --sc;
    }
  };
  std::string a, b;
  int64_t sa, sb;
  norm(*this, a, sa);
  norm(o, b, sb);
  return sa == sb && a == b;
}

std::string Decimal::str() const {
  std::string abs_int = digits.empty() ? "0" : digits;
  std::string before, after;
  if (scale >= (int64_t)abs_int.size()) {
    before = "0";
    after = std::string((size_t)scale - abs_int.size(), '0') + abs_int;
  } else {
    int64_t loc = (int64_t)abs_int.size() - scale;
    if (loc > (int64_t)abs_int.size()) {
      before = abs_int + std::string((size_t)(loc - (int64_t)abs_int.size()), '0');
    } else {
      before = abs_int.substr(0, (size_t)loc);
      after = abs_int.substr((size_t)loc);
    }
  }
  std::string s = after.empty() ? before : before + "." + after;
  return (neg && !is_zero()) ? "-" + s : s;
}

double Decimal::to_f64() const {
  if (is_zero()) return 0.0;
  std::string s = (neg ? "-" : "") + digits + "e" + std::to_string(-scale);
  return strtod(s.c_str(), nullptr);  // glibc strtod is correctly rounded
}

bool Literal::operator==(const Literal &o) const {
  if (k != o.k) return false;
  switch (k) {
    case LitKind::Integer: return mag == o.mag && positive == o.positive;
    case LitKind::Float: return dec == o.dec;
    case LitKind::String: return str == o.str;
    case LitKind::Boolean: return positive == o.positive;
    case LitKind::Interval: return interval == o.interval && unit == o.unit;
    case LitKind::Null: return true;
  }
  return false;
}

// ============================================================== helpers
namespace {

bool kw(sv s, const char *k) {  // eq_ignore_ascii_case (mod.rs:53-57)
  size_t n = strlen(k);
  if (s.size() != n) return false;
  for (size_t i = 0; i < n; ++i) {
    char c = s[i];
    if (c >= 'A' && c <= 'Z') c = (char)(c + 32);
    if (c != k[i]) return false;
  }
  return true;
}

// u128/u64/u8 FromStr and from_str_radix (literal.rs:18-31): false on empty or overflow
bool parse_uint(sv s, int radix, u128 max, u128 &out) {
  size_t i = 0;
  if (i < s.size() && s[i] == '+') ++i;  // Rust accepts a leading '+'
  if (i >= s.size()) return false;
  u128 v = 0;
  for (; i < s.size(); ++i) {
    char c = s[i];
    int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
                                             : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : 99;
    if (d >= radix) return false;
    if (v > (max - (u128)d) / (u128)radix) return false;
    v = v * (u128)radix + (u128)d;
  }
  out = v;
  return true;
}

constexpr u128 kU128Max = ~(u128)0;
constexpr u128 kU64Max = (u128)~(uint64_t)0;
constexpr u128 kU8Max = 255;

enum Power { P_Term, P_Or, P_Xor, P_And, P_Not, P_Cmp, P_Between, P_BitOr, P_BitXor, P_BitAnd, P_Shift, P_PlusMinus,
             P_MulDivMod, P_Access };  // TokenPower (mod.rs:1950-1966)
enum UPower { U_Term, U_Except, U_Union, U_Intersect };  // UnionTypePower (mod.rs:1968-1974)

Expr mk_lit(Literal &&l) {
  Expr e;
  e.k = EK::Literal;
  e.lit = std::make_unique<Literal>(std::move(l));
  return e;
}
Expr mk_bool(bool b) {
  Literal l;
  l.k = LitKind::Boolean;
  l.positive = b;
  return mk_lit(std::move(l));
}
Expr mk_null() {
  Literal l;
  l.k = LitKind::Null;
  return mk_lit(std::move(l));
}
Expr mk_un(UnOp op, Expr a) {
  Expr e;
  e.k = EK::UnaryOp;
  e.op = (uint8_t)op;
  e.kids.push_back(std::move(a));
  return e;
}
Expr mk_bin(BinOp op, Expr a, Expr b) {
  Expr e;
  e.k = EK::BinaryOp;
  e.op = (uint8_t)op;
  e.kids.reserve(2);
  e.kids.push_back(std::move(a));
  e.kids.push_back(std::move(b));
  return e;
}
Expr mk_call(FnKind f, sv name, std::vector<Expr> args) {
  Expr e;
  e.k = EK::FnCall;
  e.op = (uint8_t)f;
  e.id.name = name;
  e.kids = std::move(args);
  return e;
}
Expr mk_id(const Identifier &id) {
  Expr e;
  e.k = EK::Identifier;
  e.id = id;
  return e;
}
Expr mk_coll(CollType t, std::vector<Expr> items) {
  Expr e;
  e.k = EK::Collection;
  e.op = (uint8_t)t;
  e.kids = std::move(items);
  return e;
}
Expr mk_subquery(Query &&q) {
  Expr e;
  e.k = EK::Subquery;
  e.q = std::make_unique<Query>(std::move(q));
  return e;
}

// ---------------------------------------------------------------- simplify.rs
Expr simplified_eq(Expr l, Expr r) {  // simplify.rs:3-12
  if (l.is_lit() && r.is_lit()) return mk_bool(*l.lit == *r.lit);
  return mk_bin(BinOp::Eq, std::move(l), std::move(r));
}
Expr simplified_neq(Expr l, Expr r) {  // :14-23
  if (l.is_lit() && r.is_lit()) return mk_bool(!(*l.lit == *r.lit));
  return mk_bin(BinOp::NotEq, std::move(l), std::move(r));
}
Expr simplified_and(Expr l, Expr r) {  // :25-43
  bool b;
  if (l.is_bool_lit(&b)) return b ? std::move(r) : mk_bool(false);
  if (r.is_bool_lit(&b)) return b ? std::move(l) : mk_bool(false);
  return mk_bin(BinOp::And, std::move(l), std::move(r));
}
Expr simplified_or(Expr l, Expr r) {  // :45-63
  bool b;
  if (l.is_bool_lit(&b)) return b ? mk_bool(true) : std::move(r);
  if (r.is_bool_lit(&b)) return b ? mk_bool(true) : std::move(l);
  return mk_bin(BinOp::Or, std::move(l), std::move(r));
}
Expr simplified_xor(Expr l, Expr r) {  // :65-83
  bool b;
  if (l.is_bool_lit(&b)) return b ? mk_un(UnOp::Not, std::move(r)) : std::move(r);
  if (r.is_bool_lit(&b)) return b ? mk_un(UnOp::Not, std::move(l)) : std::move(l);
  return mk_bin(BinOp::Xor, std::move(l), std::move(r));
}
Expr simplified_not(Expr a) {  // :85-92
  bool b;
  if (a.is_bool_lit(&b)) return mk_bool(!b);
  return mk_un(UnOp::Not, std::move(a));
}
Expr simplified_is_null(Expr a) {  // :94-101
  if (a.is_lit()) return mk_bool(a.lit->k == LitKind::Null);
  return mk_un(UnOp::IsNull, std::move(a));
}
Expr simplified_is_not_null(Expr a) {  // :103-110
  if (a.is_lit()) return mk_bool(a.lit->k != LitKind::Null);
  return mk_un(UnOp::IsNotNull, std::move(a));
}

}  // namespace

// ---------------------------------------------------------------- literal.rs unescape
// Reads one code point; the input is valid UTF-8 (a token span).
static int32_t next_cp(sv s, size_t &i) {
  const unsigned char *u = (const unsigned char *)s.data();
  unsigned c = u[i];
  int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : 4;
  uint32_t cp = len == 1 ? c : len == 2 ? (c & 0x1F) : len == 3 ? (c & 0x0F) : (c & 0x07);
  for (int k = 1; k < len && i + k < s.size(); ++k) cp = (cp << 6) | (u[i + k] & 0x3F);
  i += len;
  return (int32_t)cp;
}

bool unescape(sv raw, char quote, std::string &out, ParseError &err) {
  out.clear();
  out.reserve(raw.size());
  size_t i = 0;
  while (i < raw.size()) {
    int32_t ch = next_cp(raw, i);
    if (ch == quote) {
      if (i < raw.size()) next_cp(raw, i);  // the doubled quote
      out += quote;
    } else if (ch == '\\') {
      if (i >= raw.size()) {
        // unreachable for tokenizer output (literal.rs:58-62); keep the backslash
        out += '\\';
        break;
      }
      int32_t n = next_cp(raw, i);
      if (n == 'n') {
        out += '\n';
      } else if (n == 'r') {
        out += '\r';
      } else if (n == 't') {
        out += '\t';
      } else if (n == 'u') {
        int32_t open = i < raw.size() ? next_cp(raw, i) : -1;  // consumed even if not '{'
        if (open != '{') {
          out += 'u';
          continue;
        }
        std::string hex;
        while (i < raw.size()) {
          size_t s0 = i;
          int32_t h = next_cp(raw, i);
          if (h == '}') break;
          hex.append(raw.data() + s0, i - s0);
        }
        u128 v;
        bool ok = parse_uint(hex, 16, (u128)0xFFFFFFFFu, v);
        if (ok && ((v >= 0xD800 && v <= 0xDFFF) || v > 0x10FFFF)) ok = false;  // char::from_u32
        if (!ok) {
          err.lex = false;
          err.msg = "invalid escaped unicode '\\u{" + hex + "}' in string literal";
          return false;
        }
        out += utf8_encode((int32_t)v);
      } else {
        out += utf8_encode(n);
      }
    } else {
      out += utf8_encode(ch);
    }
  }
  return true;
}

// ============================================================== the parser
namespace {

struct Fail {};  // unwinds to parse(); the message is in Parser::err

class Parser {
 public:
  explicit Parser(sv sql) : tz_(sql.data(), sql.size()) {}
  ParseError err;
  void parse_stmt(Statement &st);

 private:
  Tokenizer tz_;
  bool has_peek_ = false;
  Token peeked_;

  // ---------------------------------------------------------- errors
  [[noreturn]] void raise(bool lex, std::string msg) {
    err.lex = lex;
    err.msg = std::move(msg);
    throw Fail{};
  }
  [[noreturn]] void not_expected_types(std::initializer_list<Tok> exp, const Token &t) {
    std::string m = "expected token (";
    bool first = true;
    for (Tok e : exp) {
      if (!first) m += ", ";
      m += tok_name(e);
      first = false;
    }
    raise(false, m + ") but found token " + tok_name(t.t) + " at " + pos(t).str());
  }
  [[noreturn]] void not_expected_kw(std::initializer_list<const char *> exp, sv actual, const Token &t) {
    std::string m = "expected keyword (";
    bool first = true;
    for (const char *e : exp) {
      if (!first) m += ", ";
      m += e;
      first = false;
    }
    raise(false, m + ") but found token " + std::string(actual) + " at " + pos(t).str());
  }
  [[noreturn]] void parse_fail(const char *msg, const Token &t) {
    raise(false, std::string("fail to parse (") + msg + ") at " + pos(t).str());
  }
  [[noreturn]] void conflicts(const std::string &a, const std::string &b, const Token &t) {
    raise(false, "(" + a + ") conflicts with (" + b + ") near " + pos(t).str());
  }

  // ---------------------------------------------------------- token stream (mod.rs:1852-1893)
  Token lex_one() {
    Token t;
    LexError le;
    for (;;) {
      if (!tz_.next_token(t, le)) raise(true, le.str());
      if (!t.is_whitespace()) return t;
    }
  }
  const Token &peek() {
    if (!has_peek_) {
      peeked_ = lex_one();
      has_peek_ = true;
    }
    return peeked_;
  }
  void consume_peeked() { has_peek_ = false; }
  Token next() {
    if (has_peek_) {
      has_peek_ = false;
      return peeked_;
    }
    return lex_one();
  }
  sv str(const Token &t) const { return sv(tz_.source().data() + t.span.start, t.span.end - t.span.start); }
  Position pos(const Token &t) const { return tz_.source().pos_at(t.span.start); }

  Token next_expect(std::initializer_list<Tok> exp) {
    Token t = next();
    for (Tok e : exp)
      if (t.t == e) return t;
    not_expected_types(exp, t);
  }
  bool next_if(Tok e) {
    if (peek().t == e) {
      consume_peeked();
      return true;
    }
    return false;
  }

  // ---------------------------------------------------------- keywords (mod.rs:1621-1686)
  bool try_kw(const char *k) {
    const Token &t = peek();
    if (!t.maybe_keyword()) return false;
    if (kw(str(t), k)) {
      consume_peeked();
      return true;
    }
    return false;
  }
  void must_kw(const char *k) {
    Token t = next_expect({Tok::KeywordOrIdentifier});
    if (!kw(str(t), k)) not_expected_kw({k}, str(t), t);
  }
  int must_one_of(std::initializer_list<const char *> ks) {
    Token t = next_expect({Tok::KeywordOrIdentifier});
    sv s = str(t);
    int i = 0;
    for (const char *k : ks) {
      if (kw(s, k)) return i;
      ++i;
    }
    not_expected_kw(ks, s, t);
  }
  void must_kws(std::initializer_list<const char *> ks) {
    for (const char *k : ks) must_kw(k);
  }
  sv must_ident_string() {
    Token t = next_expect({Tok::KeywordOrIdentifier, Tok::DelimitedIdentifier});
    return str(t);
  }
  bool peek_is_kw(const char *k) {
    const Token &t = peek();
    return !t.is_terminator() && t.maybe_keyword() && kw(str(t), k);
  }

  // ---------------------------------------------------------- literals (mod.rs:1815-1849)
  u128 integer_literal(u128 max) {
    Token t = next_expect({Tok::IntegerLiteral, Tok::HexLiteral});
    return integer_of(t, max);
  }
  u128 integer_of(const Token &t, u128 max) {
    sv s = str(t);
    u128 v = 0;
    if (t.t == Tok::IntegerLiteral) {
      if (!parse_uint(s, 10, max, v)) raise(false, "invalid integer '" + std::string(s) + "'");
    } else {
      if (!parse_uint(s, 16, max, v)) raise(false, "invalid hex '0x" + std::string(s) + "'");
    }
    return v;
  }
  Decimal decimal_of(sv s) {
    Decimal d;
    size_t dot = s.find('.');
    std::string digits = dot == sv::npos ? std::string(s) : std::string(s.substr(0, dot)) + std::string(s.substr(dot + 1));
    d.scale = dot == sv::npos ? 0 : (int64_t)(s.size() - dot - 1);
    d.digits = strip_zeros(digits);
    return d;
  }
  std::string string_literal() {
    Token t = next_expect({Tok::RawStringLiteral, Tok::EscapedSQStringLiteral, Tok::EscapedDQStringLiteral});
    return string_of(t);
  }
  std::string string_of(const Token &t) {
    sv s = str(t);
    if (t.t == Tok::RawStringLiteral) return std::string(s);
    std::string out;
    if (!unescape(s, t.t == Tok::EscapedSQStringLiteral ? '\'' : '"', out, err)) throw Fail{};
    return out;
  }

  // ---------------------------------------------------------- statements
  bool try_select(sv k, Statement &st);
  bool try_insert(sv k, Statement &st);
  bool try_explain(sv k, Statement &st);
  bool try_alter(sv k, Statement &st);
  bool try_create(sv k, Statement &st);
  bool try_describe(sv k, Statement &st);
  bool try_drop(sv k, Statement &st, bool truncate);
  bool try_optimize(sv k, Statement &st);
  bool try_set(sv k, Statement &st);

  // ---------------------------------------------------------- queries
  Query subquery() { return subquery_tdop(U_Term); }
  Query subquery_tdop(int power);
  Query query_tdop(bool with, int power);
  std::unique_ptr<QueryBody> query_body(bool with);
  std::vector<CTE> clause_with();
  QuerySource query_source();
  QueryExpr query_expr();
  std::vector<QueryExpr> query_expr_list();
  bool clause_join(JoinClause &j);
  int union_power(const Token &t) {
    if (t.t != Tok::KeywordOrIdentifier) return U_Term;
    sv s = str(t);
    if (kw(s, "union")) return U_Union;
    if (kw(s, "intersect")) return U_Intersect;
    if (kw(s, "except")) return U_Except;
    return U_Term;
  }

  // ---------------------------------------------------------- DDL
  TableDef table_def();
  ViewDef view_def();
  ColumnDef column_def();
  ConstraintDef constraint_def();
  IndexDef index_def();
  DataType datatype();

  // ---------------------------------------------------------- expressions
  std::vector<Expr> expr_list() {
    std::vector<Expr> v;
    do v.push_back(expr()); while (next_if(Tok::Comma));
    return v;
  }
  Expr expr() { return expr_tdop(P_Term); }
  Expr expr_tdop(int power) {
    Expr e = prefix();
    for (;;) {
      int np = token_power(peek());
      if (np <= power) break;
      e = infix(std::move(e), np);
    }
    return e;
  }
  Expr prefix();
  Expr infix(Expr left, int power);
  Identifier ident_based_prefix(sv prefix);
  Identifier must_identifier();
  bool fn_call_args(std::vector<Expr> &args);
  Expr if_body();
  Expr case_when_body();
  int token_power(const Token &t) {
    switch (t.t) {
      case Tok::Eq:
      case Tok::NotEq:
      case Tok::Lt:
      case Tok::LtEq:
      case Tok::GtEq:
      case Tok::Gt: return P_Cmp;
      case Tok::BitOr: return P_BitOr;
      case Tok::BitXor: return P_BitXor;
      case Tok::BitAnd: return P_BitAnd;
      case Tok::BitLShift:
      case Tok::BitRShift: return P_Shift;
      case Tok::Plus:
      case Tok::Minus: return P_PlusMinus;
      case Tok::Mul:
      case Tok::Div:
      case Tok::Mod: return P_MulDivMod;
      case Tok::LBracket: return P_Access;
      case Tok::KeywordOrIdentifier: {
        sv s = str(t);
        if (kw(s, "or")) return P_Or;
        if (kw(s, "xor")) return P_Xor;
        if (kw(s, "and")) return P_And;
        if (kw(s, "not")) return P_Not;
        if (kw(s, "is") || kw(s, "in") || kw(s, "like") || kw(s, "ilike")) return P_Cmp;
        if (kw(s, "between")) return P_Between;
        return P_Term;
      }
      default: return P_Term;
    }
  }
};

// ============================================================== statement dispatch (mod.rs:128-180)
void Parser::parse_stmt(Statement &st) {
  Token t = next();
  if (t.is_terminator()) raise(false, "empty query");
  if (!t.maybe_keyword()) parse_fail("statements should start with a keyword", t);
  sv k = str(t);
  bool ok = try_select(k, st) || try_insert(k, st) || try_explain(k, st) || try_alter(k, st) ||
            try_create(k, st) || try_describe(k, st) || try_drop(k, st, false) || try_drop(k, st, true) ||
            try_optimize(k, st) || try_set(k, st);
  if (!ok) parse_fail("cannot recognize statement", t);
  const Token &p = peek();
  if (!p.is_terminator()) parse_fail("more than one statement", p);
}

bool Parser::try_select(sv k, Statement &st) {  // mod.rs:190-203
  bool with = kw(k, "with");
  if (!with && !kw(k, "select")) return false;
  st.k = StmtKind::Select;
  st.query = query_tdop(with, U_Term);
  return true;
}

bool Parser::try_explain(sv k, Statement &st) {  // mod.rs:674-686
  if (!kw(k, "explain")) return false;
  st.k = StmtKind::Explain;
  st.query = subquery();
  return true;
}

bool Parser::try_insert(sv k, Statement &st) {  // mod.rs:589-670
  if (!kw(k, "insert")) return false;
  must_kw("into");
  auto ins = std::make_unique<InsertStmt>();
  ins->table = must_ident_string();
  if (next_if(Tok::LParen)) {
    std::vector<sv> cols;
    do cols.push_back(must_ident_string()); while (next_if(Tok::Comma));
    next_expect({Tok::RParen});
    ins->columns = std::move(cols);
  }
  Token report = peek();
  switch (must_one_of({"values", "from", "select", "with"})) {
    case 0: {
      ins->k = InsertKind::Rows;
      next_expect({Tok::LParen});
      uint64_t column_size = 0;
      do {
        ins->data.push_back(expr());
        ++column_size;
      } while (next_if(Tok::Comma));
      next_expect({Tok::RParen});
      if (next_if(Tok::Comma)) {
        do {
          next_expect({Tok::LParen});
          uint64_t this_size = 0;
          do {
            ins->data.push_back(expr());
            ++this_size;
          } while (next_if(Tok::Comma));
          if (this_size != column_size) {
            Token r = peek();
            conflicts("row has " + std::to_string(this_size) + " column(s)",
                      "previous rows have " + std::to_string(column_size) + " column(s)", r);
          }
          next_expect({Tok::RParen});
        } while (next_if(Tok::Comma));
      }
      ins->column_size = column_size;
      break;
    }
    case 1: {
      Expr e = expr();
      if (e.k != EK::FnCall) parse_fail("insert source must be a subquery, values, or a function call", report);
      ins->k = InsertKind::FnCall;
      ins->fn = std::move(e);
      break;
    }
    case 2:
      ins->k = InsertKind::Subquery;
      ins->query = query_tdop(false, U_Term);
      break;
    default:
      ins->k = InsertKind::Subquery;
      ins->query = query_tdop(true, U_Term);
      break;
  }
  st.k = StmtKind::Insert;
  st.insert = std::move(ins);
  return true;
}

bool Parser::try_create(sv k, Statement &st) {  // mod.rs:689-710
  if (!kw(k, "create")) return false;
  int idx = must_one_of({"table", "view"});
  bool ine = false;
  if (try_kw("if")) {
    must_kws({"not", "exists"});
    ine = true;
  }
  st.k = StmtKind::Create;
  st.if_flag = ine;
  st.is_view = idx == 1;
  if (idx == 0)
    st.table = std::make_unique<TableDef>(table_def());
  else
    st.view = std::make_unique<ViewDef>(view_def());
  return true;
}

TableDef Parser::table_def() {  // mod.rs:712-805
  TableDef d;
  d.name = must_ident_string();
  next_expect({Tok::LParen});
  do {
    if (try_kw("index"))
      d.indexes.push_back(index_def());
    else if (try_kw("constraint"))
      d.constraints.push_back(constraint_def());
    else
      d.columns.push_back(column_def());
  } while (next_if(Tok::Comma));
  next_expect({Tok::RParen});
  for (;;) {
    Token t = peek();
    if (!t.maybe_keyword()) break;
    switch (must_one_of({"primary", "order", "partition", "comment"})) {
      case 0:
        if (d.primary_key) conflicts("primary key", "primary key", t);
        must_kw("key");
        d.primary_key = expr_list();
        break;
      case 1:
        if (d.order_by) conflicts("order by", "order by", t);
        must_kw("by");
        d.order_by = expr_list();
        break;
      case 2:
        if (d.partition_by) conflicts("partition by", "partition by", t);
        must_kw("by");
        d.partition_by = expr();
        break;
      default:
        if (d.comment) conflicts("comment", "comment", t);
        d.comment = string_literal();
        break;
    }
  }
  return d;
}

ViewDef Parser::view_def() {  // mod.rs:807-911
  ViewDef d;
  d.name = must_ident_string();
  bool has_strategy = false;
  for (;;) {
    Token t = peek();
    int i = must_one_of({"as", "update", "primary", "order", "partition", "comment"});
    if (i == 0) {
      if (!has_strategy) not_expected_kw({"update"}, "as", t);
      break;
    }
    switch (i) {
      case 1:
        if (has_strategy) conflicts("update by", "update by", t);
        must_kw("by");
        d.strategy = must_ident_string();
        has_strategy = true;
        break;
      case 2:
        if (d.primary_key) conflicts("primary key", "primary key", t);
        must_kw("key");
        d.primary_key = expr_list();
        break;
      case 3:
        if (d.order_by) conflicts("order by", "order by", t);
        must_kw("by");
        d.order_by = expr_list();
        break;
      case 4:
        if (d.partition_by) conflicts("partition by", "partition by", t);
        must_kw("by");
        d.partition_by = expr();
        break;
      default:
        if (d.comment) conflicts("comment", "comment", t);
        d.comment = string_literal();
        break;
    }
  }
  d.query = subquery();
  return d;
}

ConstraintDef Parser::constraint_def() {  // mod.rs:913-918
  ConstraintDef c;
  c.name = must_ident_string();
  must_kw("check");
  c.check = expr();
  return c;
}

IndexDef Parser::index_def() {  // mod.rs:920-934
  IndexDef d;
  d.name = must_ident_string();
  Token report = peek();
  Expr e = expr();
  if (e.k != EK::FnCall) parse_fail("indexer must be a function call", report);
  d.indexer = std::move(e);
  return d;
}

ColumnDef Parser::column_def() {  // mod.rs:936-972
  ColumnDef c;
  c.name = must_ident_string();
  c.t = datatype();
  for (;;) {
    Token t = peek();
    if (!t.maybe_keyword()) break;
    if (must_one_of({"default", "comment"}) == 0) {
      if (c.default_) conflicts("default", "default", t);
      c.default_ = expr();
    } else {
      if (c.comment) conflicts("comment", "comment", t);
      c.comment = string_literal();
    }
  }
  return c;
}

DataType Parser::datatype() {  // mod.rs:1688-1797
  static const Scalar simple[] = {Scalar::Int8,     Scalar::Int16,     Scalar::Int32,      Scalar::Int64,
                                  Scalar::Int128,   Scalar::UInt8,     Scalar::UInt16,     Scalar::UInt32,
                                  Scalar::UInt64,   Scalar::UInt128,   Scalar::Serial32,   Scalar::Serial64,
                                  Scalar::Serial128, Scalar::USerial32, Scalar::USerial64, Scalar::USerial128};
  int i = must_one_of({"int8", "int16", "int32", "int64", "int128", "uint8", "uint16", "uint32", "uint64",
                       "uint128", "serial32", "serial64", "serial128", "userial32", "userial64", "userial128",
                       "decimal32", "decimal64", "float32", "float64", "boolean", "chars", "string", "uuid", "date",
                       "datetime", "array", "enum", "tuple", "map", "dictionary", "nullable"});
  DataType d;
  if (i < 16) {
    d.s = simple[i];
    return d;
  }
  switch (i) {
    case 16:
    case 17:
      next_expect({Tok::LParen});
      d.s = i == 16 ? Scalar::Decimal32 : Scalar::Decimal64;
      d.param = (uint64_t)integer_literal(kU8Max);
      next_expect({Tok::RParen});
      return d;
    case 18: d.s = Scalar::Float32; return d;
    case 19: d.s = Scalar::Float64; return d;
    case 20: d.s = Scalar::Boolean; return d;
    case 21:
      next_expect({Tok::LParen});
      d.s = Scalar::Chars;
      d.param = (uint64_t)integer_literal(kU64Max);
      next_expect({Tok::RParen});
      return d;
    case 22:
      d.s = Scalar::String;
      if (peek().t == Tok::LParen) {
        next_expect({Tok::LParen});
        d.param = (uint64_t)integer_literal(kU64Max);
        next_expect({Tok::RParen});
      }
      return d;
    case 23: d.s = Scalar::Uuid; return d;
    case 24: d.s = Scalar::Date; return d;
    case 25: d.s = Scalar::Datetime; return d;
    default: break;
  }
  d.scalar = false;
  next_expect({Tok::LParen});
  switch (i) {
    case 26:
      d.c = Compound::Array;
      d.kids.push_back(datatype());
      break;
    case 27: {
      d.c = Compound::Enum;
      uint64_t id = 0;
      do {
        EnumBind b;
        b.literal = string_literal();
        if (next_if(Tok::Eq)) id = (uint64_t)integer_literal(kU64Max);
        b.id = id;
        d.binds.push_back(std::move(b));
        id += 1;  // usize add; the reference panics on overflow in debug builds only
      } while (next_if(Tok::Comma));
      break;
    }
    case 28:
      d.c = Compound::Tuple;
      do d.kids.push_back(datatype()); while (next_if(Tok::Comma));
      break;
    case 29: {
      d.c = Compound::Map;
      DataType key = datatype();
      next_expect({Tok::Comma});
      DataType value = datatype();
      d.kids.push_back(std::move(value));  // stored as (value, key), mod.rs:1780
      d.kids.push_back(std::move(key));
      break;
    }
    case 30:
      d.c = Compound::Dictionary;
      d.kids.push_back(datatype());
      break;
    default:
      d.c = Compound::Nullable;
      d.kids.push_back(datatype());
      break;
  }
  next_expect({Tok::RParen});
  return d;
}

bool Parser::try_alter(sv k, Statement &st) {  // mod.rs:976-1059
  if (!kw(k, "alter")) return false;
  must_kw("table");
  auto a = std::make_unique<AlterStmt>();
  a->table = must_ident_string();
  switch (must_one_of({"add", "drop", "rename"})) {
    case 0: {
      a->k = AlterKind::Add;
      if (try_kw("if")) {
        must_kws({"not", "exists"});
        a->if_flag = true;
      }
      switch (must_one_of({"column", "index", "constraint"})) {
        case 0: a->entity = EntityKind::Column; a->column = column_def(); break;
        case 1: a->entity = EntityKind::Index; a->index = index_def(); break;
        default: a->entity = EntityKind::Constraint; a->constraint = constraint_def(); break;
      }
      if (try_kw("first")) {
        a->pos = Position_::First;
      } else if (try_kw("after")) {
        a->pos = Position_::After;
        a->after = must_ident_string();
      } else {
        a->pos = Position_::Last;
      }
      break;
    }
    case 1: {
      a->k = AlterKind::Drop;
      if (try_kw("if")) {
        must_kw("exists");
        a->if_flag = true;
      }
      switch (must_one_of({"column", "index", "constraint", "partition"})) {
        case 0: a->entity = EntityKind::Column; a->name = must_ident_string(); break;
        case 1: a->entity = EntityKind::Index; a->name = must_ident_string(); break;
        case 2: a->entity = EntityKind::Constraint; a->name = must_ident_string(); break;
        default: a->entity = EntityKind::Partition; a->partition = string_literal(); break;
      }
      break;
    }
    default: {
      a->k = AlterKind::Rename;
      switch (must_one_of({"column", "index", "constraint", "table"})) {
        case 0: a->entity = EntityKind::Column; a->name = must_ident_string(); break;
        case 1: a->entity = EntityKind::Index; a->name = must_ident_string(); break;
        case 2: a->entity = EntityKind::Constraint; a->name = must_ident_string(); break;
        default: a->entity = EntityKind::Table; break;
      }
      a->new_name = must_ident_string();
      break;
    }
  }
  st.k = StmtKind::Alter;
  st.alter = std::move(a);
  return true;
}

bool Parser::try_describe(sv k, Statement &st) {  // mod.rs:1063-1079
  if (!kw(k, "describe")) return false;
  st.k = StmtKind::Describe;
  switch (must_one_of({"table", "view", "database"})) {
    case 0: st.describe = DescribeKind::Table; st.name = must_ident_string(); break;
    case 1: st.describe = DescribeKind::View; st.name = must_ident_string(); break;
    default: st.describe = DescribeKind::Database; break;
  }
  return true;
}

bool Parser::try_drop(sv k, Statement &st, bool truncate) {  // mod.rs:1083-1142
  if (!kw(k, truncate ? "truncate" : "drop")) return false;
  st.k = truncate ? StmtKind::Truncate : StmtKind::Drop;
  st.is_view = must_one_of({"table", "view"}) == 1;
  if (try_kw("if")) {
    must_kw("exists");
    st.if_flag = true;
  }
  st.name = must_ident_string();
  return true;
}

bool Parser::try_optimize(sv k, Statement &st) {  // mod.rs:1146-1172
  if (!kw(k, "optimize")) return false;
  must_kw("table");
  st.k = StmtKind::Optimize;
  st.name = must_ident_string();
  if (peek().is_terminator()) return true;
  must_kws({"on", "partition"});
  st.value = expr();
  return true;
}

bool Parser::try_set(sv k, Statement &st) {  // mod.rs:1176-1196
  if (!kw(k, "set")) return false;
  Token t = next_expect({Tok::ConfigIdentifier});
  st.k = StmtKind::Set;
  st.name = str(t);
  next_expect({Tok::Eq});
  st.value = expr();
  return true;
}

// ============================================================== queries (mod.rs:205-586)
Query Parser::subquery_tdop(int power) {
  bool paren = next_if(Tok::LParen);
  bool with = must_one_of({"with", "select"}) == 0;
  Query q = query_tdop(with, paren ? U_Term : power);
  if (paren) next_expect({Tok::RParen});
  return q;
}

Query Parser::query_tdop(bool with, int power) {
  Query q;
  q.body = query_body(with);
  for (;;) {
    int np = union_power(peek());
    if (np <= power) break;
    consume_peeked();
    UnionType ut;
    if (np == U_Intersect)
      ut = UnionType::Intersect;
    else if (np == U_Union)
      ut = must_one_of({"all", "distinct"}) == 0 ? UnionType::UnionAll : UnionType::UnionDistinct;
    else
      ut = UnionType::Except;
    Query u;
    u.is_union = true;
    u.ut = ut;
    u.l = std::make_unique<Query>(std::move(q));
    u.r = std::make_unique<Query>(subquery_tdop(np));
    q = std::move(u);
  }
  return q;
}

std::unique_ptr<QueryBody> Parser::query_body(bool with) {
  auto b = std::make_unique<QueryBody>();
  if (with) {
    b->with = clause_with();
    must_kw("select");
  }
  if (try_kw("distinct")) {
    b->distinct = true;
    if (try_kw("on")) {
      next_expect({Tok::LParen});
      b->distinct_on = query_expr_list();
      next_expect({Tok::RParen});
    }
  }
  b->columns = query_expr_list();
  if (peek_is_kw("from")) {
    consume_peeked();
    b->from = query_source();
  }
  for (;;) {
    JoinClause j;
    if (!clause_join(j)) break;
    b->joins.push_back(std::move(j));
  }
  if (peek_is_kw("where")) {
    consume_peeked();
    b->where = expr();
  }
  if (peek_is_kw("group")) {
    consume_peeked();
    must_kw("by");
    b->group_by = query_expr_list();
  }
  if (peek_is_kw("having")) {
    consume_peeked();
    b->having = expr();
  }
  if (peek_is_kw("order")) {  // mod.rs:476-501
    consume_peeked();
    must_kw("by");
    std::vector<OrderKey> keys;
    do {
      OrderKey k;
      k.e = query_expr();
      if (try_kw("desc")) {
        k.desc = true;
      } else {
        try_kw("desc");  // the reference tests DESC twice; ASC is never consumed
        k.desc = false;
      }
      keys.push_back(std::move(k));
    } while (next_if(Tok::Comma));
    b->order_by = std::move(keys);
  }
  if (peek_is_kw("limit")) {  // mod.rs:503-544
    consume_peeked();
    LimitClause l;
    uint64_t first = (uint64_t)integer_literal(kU64Max);
    const Token &t = peek();
    if (t.t == Tok::Comma) {
      consume_peeked();
      l.size = (uint64_t)integer_literal(kU64Max);
      l.offset = first;
    } else if (t.t == Tok::KeywordOrIdentifier && kw(str(t), "offset")) {
      consume_peeked();
      l.size = first;
      l.offset = (uint64_t)integer_literal(kU64Max);
    } else {
      l.size = first;
      l.offset = 0;
    }
    if (try_kw("with")) {
      must_kw("ties");
      l.with_ties = true;
    }
    b->limit = l;
  }
  return b;
}

std::vector<CTE> Parser::clause_with() {  // mod.rs:327-347
  std::vector<CTE> list;
  do {
    CTE c;
    c.alias = must_ident_string();
    must_kw("as");
    Token report = peek();
    Expr e = expr();
    if (e.k != EK::Subquery) parse_fail("not a subquery", report);
    c.q = std::move(e.q);
    list.push_back(std::move(c));
  } while (next_if(Tok::Comma));
  return list;
}

bool Parser::clause_join(JoinClause &j) {  // mod.rs:376-431
  const Token &t = peek();
  if (t.is_terminator() || !t.maybe_keyword()) return false;
  sv s = str(t);
  if (kw(s, "inner")) {
    consume_peeked();
    j.t = JoinType::Inner;
  } else if (kw(s, "full")) {
    consume_peeked();
    try_kw("outer");
    j.t = JoinType::FullOuter;
  } else if (kw(s, "left") || kw(s, "right")) {
    bool left = kw(s, "left");
    consume_peeked();
    if (try_kw("semi")) {
      j.t = left ? JoinType::LeftSemi : JoinType::RightSemi;
    } else if (try_kw("anti")) {
      j.t = left ? JoinType::LeftAnti : JoinType::RightAnti;
    } else {
      try_kw("outer");
      j.t = left ? JoinType::LeftOuter : JoinType::RightOuter;
    }
  } else if (kw(s, "join")) {
    j.t = JoinType::Inner;
  } else {
    return false;
  }
  must_kw("join");
  j.src = query_source();
  if (must_one_of({"on", "using"}) == 0) {
    j.on = true;
    j.cond = expr();
  } else {
    j.on = false;
    next_expect({Tok::LParen});
    do j.using_.push_back(must_identifier()); while (next_if(Tok::Comma));
    next_expect({Tok::RParen});
  }
  return true;
}

QuerySource Parser::query_source() {  // mod.rs:546-569
  Token report = peek();
  Expr e = expr();
  QuerySource s;
  if (e.k == EK::Subquery) {
    s.k = SourceKind::Subquery;
    s.e = std::move(e);
  } else if (e.k == EK::FnCall) {
    s.k = SourceKind::TableFn;
    s.e = std::move(e);
  } else if (e.k == EK::Identifier && !e.id.wildcard) {
    s.k = SourceKind::Table;
    s.table = e.id.name;
  } else {
    parse_fail("query source must be a subquery, a table function or a table", report);
  }
  if (try_kw("as")) s.alias = must_ident_string();
  return s;
}

QueryExpr Parser::query_expr() {  // mod.rs:571-579
  QueryExpr q;
  q.e = expr();
  if (try_kw("as")) q.alias = must_ident_string();
  return q;
}

std::vector<QueryExpr> Parser::query_expr_list() {
  std::vector<QueryExpr> v;
  do v.push_back(query_expr()); while (next_if(Tok::Comma));
  return v;
}

// ============================================================== expressions (mod.rs:1198-1619)
Expr Parser::prefix() {
  Token t = next();
  sv s = str(t);
  switch (t.t) {
    case Tok::LParen: {
      const Token &p = peek();
      Expr e;
      if (p.maybe_keyword() && (kw(str(p), "select") || kw(str(p), "with"))) {
        e = mk_subquery(subquery());
      } else {
        std::vector<Expr> v = expr_list();
        if (v.size() == 1)
          e = std::move(v[0]);
        else
          e = mk_coll(CollType::Tuple, std::move(v));
      }
      next_expect({Tok::RParen});
      return e;
    }
    case Tok::LBracket: {
      Expr e = mk_coll(CollType::Array, expr_list());
      next_expect({Tok::RBracket});
      return e;
    }
    case Tok::LBrace: {
      std::vector<Expr> items;
      do {
        items.push_back(expr());
        next_expect({Tok::Colon});
        items.push_back(expr());
      } while (next_if(Tok::Comma));
      Expr e = mk_coll(CollType::Map, std::move(items));
      next_expect({Tok::RBrace});
      return e;
    }
    case Tok::Minus: {  // '-' only before a numeric literal (mod.rs:1259-1269)
      Token n = next_expect({Tok::IntegerLiteral, Tok::HexLiteral, Tok::FloatLiteral});
      Literal l;
      if (n.t == Tok::FloatLiteral) {
        l.k = LitKind::Float;
        l.dec = decimal_of(str(n));
        l.dec.neg = !l.dec.is_zero();
      } else {
        l.k = LitKind::Integer;
        l.mag = integer_of(n, kU128Max);
        l.positive = false;
      }
      return mk_lit(std::move(l));
    }
    case Tok::Plus: return prefix();
    case Tok::Mul: {
      Identifier id;
      id.wildcard = true;
      return mk_id(id);
    }
    case Tok::BitNot: return mk_un(UnOp::BitwiseNot, prefix());
    case Tok::RawStringLiteral:
    case Tok::EscapedSQStringLiteral:
    case Tok::EscapedDQStringLiteral: {
      Literal l;
      l.k = LitKind::String;
      l.str = string_of(t);
      return mk_lit(std::move(l));
    }
    case Tok::FloatLiteral: {
      Literal l;
      l.k = LitKind::Float;
      l.dec = decimal_of(s);
      return mk_lit(std::move(l));
    }
    case Tok::HexLiteral:
    case Tok::IntegerLiteral: {
      Literal l;
      l.k = LitKind::Integer;
      l.mag = integer_of(t, kU128Max);
      l.positive = true;
      return mk_lit(std::move(l));
    }
    case Tok::KeywordOrIdentifier: {
      if (kw(s, "true")) return mk_bool(true);
      if (kw(s, "false")) return mk_bool(false);
      if (kw(s, "null")) return mk_null();
      if (kw(s, "not")) return simplified_not(prefix());
      if (kw(s, "interval")) {  // mod.rs:1489-1503
        Literal l;
        l.k = LitKind::Interval;
        l.interval = (uint64_t)integer_literal(kU64Max);
        l.unit = (IntervalUnit)must_one_of({"second", "minute", "hour", "day", "month", "year"});
        return mk_lit(std::move(l));
      }
      if (kw(s, "if")) return if_body();
      if (kw(s, "case")) return case_when_body();
      std::vector<Expr> args;
      if (fn_call_args(args)) return mk_call(FnKind::Others, s, std::move(args));
      return mk_id(ident_based_prefix(s));
    }
    case Tok::DelimitedIdentifier: return mk_id(ident_based_prefix(s));
    case Tok::QueryParameter: {
      Expr e;
      e.k = EK::QueryParameter;
      e.param = (uint64_t)integer_literal(kU64Max);  // A8(ii): a further integer is demanded
      return e;
    }
    default:
      not_expected_types({Tok::RawStringLiteral, Tok::EscapedSQStringLiteral, Tok::EscapedDQStringLiteral,
                          Tok::FloatLiteral, Tok::HexLiteral, Tok::IntegerLiteral, Tok::QueryParameter,
                          Tok::KeywordOrIdentifier, Tok::DelimitedIdentifier, Tok::LParen, Tok::LBracket,
                          Tok::LBrace, Tok::Minus, Tok::Plus, Tok::BitNot, Tok::Mul},
                         t);
  }
}

Expr Parser::infix(Expr left, int power) {
  Token t = next();
  auto bin = [&](BinOp op) { return mk_bin(op, std::move(left), expr_tdop(power)); };
  switch (t.t) {
    case Tok::Plus: return bin(BinOp::Plus);
    case Tok::Minus: return bin(BinOp::Minus);
    case Tok::Mul: return bin(BinOp::Multi);
    case Tok::Div: return bin(BinOp::Div);
    case Tok::Mod: return bin(BinOp::Mod);
    case Tok::Gt: return bin(BinOp::Gt);
    case Tok::Lt: return bin(BinOp::Lt);
    case Tok::GtEq: return bin(BinOp::GtEq);
    case Tok::LtEq: return bin(BinOp::LtEq);
    case Tok::Eq: {
      Expr r = expr_tdop(power);
      return simplified_eq(std::move(left), std::move(r));
    }
    case Tok::NotEq: {
      Expr r = expr_tdop(power);
      return simplified_neq(std::move(left), std::move(r));
    }
    case Tok::BitOr: return bin(BinOp::BitwiseOr);
    case Tok::BitAnd: return bin(BinOp::BitwiseAnd);
    case Tok::BitXor: return bin(BinOp::BitwiseXor);
    case Tok::BitLShift: return bin(BinOp::BitwiseLeftShift);
    case Tok::BitRShift: return bin(BinOp::BitwiseRightShift);
    case Tok::LBracket: {
      Expr e = expr();
      next_expect({Tok::RBracket});
      return mk_bin(BinOp::IndexAccess, std::move(left), std::move(e));
    }
    case Tok::KeywordOrIdentifier: break;
    default: raise(false, "internal error: unexpected infix token");  // unreachable!() in the reference
  }
  if (power == P_And) {
    Expr r = expr_tdop(power);
    return simplified_and(std::move(left), std::move(r));
  }
  if (power == P_Or) {
    Expr r = expr_tdop(power);
    return simplified_or(std::move(left), std::move(r));
  }
  if (power == P_Xor) {
    Expr r = expr_tdop(power);
    return simplified_xor(std::move(left), std::move(r));
  }
  if (power == P_Not) {  // `x NOT IN/LIKE/ILIKE/BETWEEN/EXISTS` (mod.rs:1399-1427)
    switch (must_one_of({"in", "like", "ilike", "between", "exists"})) {
      case 0: return mk_bin(BinOp::NotIn, std::move(left), expr_tdop(P_Cmp));
      case 1: return mk_bin(BinOp::NotLike, std::move(left), expr_tdop(P_Cmp));
      case 2: return mk_bin(BinOp::NotILike, std::move(left), expr_tdop(P_Cmp));
      case 3: {
        Expr lo = expr_tdop(P_Between);
        must_kw("and");
        Expr hi = expr_tdop(P_Between);
        std::vector<Expr> a;
        a.push_back(std::move(left));
        a.push_back(std::move(lo));
        a.push_back(std::move(hi));
        return mk_call(FnKind::NotBetween, sv(), std::move(a));
      }
      default: {
        std::vector<Expr> a;
        if (!fn_call_args(a)) parse_fail("`not exists` should have arguments", t);
        return mk_call(FnKind::NotExists, sv(), std::move(a));
      }
    }
  }
  sv s = str(t);
  if (kw(s, "is")) {
    if (must_one_of({"not", "null"}) == 0) {
      must_kw("null");
      return simplified_is_not_null(std::move(left));
    }
    return simplified_is_null(std::move(left));
  }
  if (kw(s, "in")) return bin(BinOp::In);
  if (kw(s, "like")) return bin(BinOp::Like);
  if (kw(s, "ilike")) return bin(BinOp::ILike);
  if (kw(s, "between")) {
    Expr lo = expr_tdop(P_Between);
    must_kw("and");
    Expr hi = expr_tdop(P_Between);
    std::vector<Expr> a;
    a.push_back(std::move(left));
    a.push_back(std::move(lo));
    a.push_back(std::move(hi));
    return mk_call(FnKind::Between, sv(), std::move(a));
  }
  if (kw(s, "exists")) {
    std::vector<Expr> a;
    if (!fn_call_args(a)) parse_fail("`exists` should have arguments", t);
    return mk_call(FnKind::Exists, sv(), std::move(a));
  }
  not_expected_kw({"and", "or", "xor", "not", "is", "in", "like", "ilike", "between", "exists"}, s, t);
}

Identifier Parser::ident_based_prefix(sv prefix) {  // mod.rs:1506-1523
  Identifier id;
  if (next_if(Tok::Dot)) {
    Token t = next_expect({Tok::DelimitedIdentifier, Tok::KeywordOrIdentifier, Tok::Mul});
    id.qualified = true;
    id.qualifier = prefix;
    if (t.t == Tok::Mul)
      id.wildcard = true;
    else
      id.name = str(t);
  } else {
    id.name = prefix;
  }
  return id;
}

Identifier Parser::must_identifier() {  // mod.rs:1525-1532
  Token t = next_expect({Tok::DelimitedIdentifier, Tok::KeywordOrIdentifier, Tok::Mul});
  if (t.t == Tok::Mul) {
    Identifier id;
    id.wildcard = true;
    return id;
  }
  return ident_based_prefix(str(t));
}

bool Parser::fn_call_args(std::vector<Expr> &args) {  // mod.rs:1534-1556
  if (!next_if(Tok::LParen)) return false;
  const Token &t = peek();
  if (t.t == Tok::RParen) {
    consume_peeked();
    return true;
  }
  if (t.t == Tok::KeywordOrIdentifier && (kw(str(t), "select") || kw(str(t), "with"))) {
    Query q = subquery();
    next_expect({Tok::RParen});
    args.push_back(mk_subquery(std::move(q)));
    return true;
  }
  args = expr_list();
  next_expect({Tok::RParen});
  return true;
}

Expr Parser::if_body() {  // mod.rs:1571-1582
  std::vector<Expr> a;
  a.push_back(expr());
  must_kw("then");
  a.push_back(expr());
  must_kw("else");
  a.push_back(expr());
  must_kw("end");
  return mk_call(FnKind::If, sv(), std::move(a));
}

Expr Parser::case_when_body() {  // mod.rs:1585-1618
  std::vector<Expr> a;
  FnKind f;
  if (try_kw("when")) {
    f = FnKind::MultiIf;
  } else {
    a.push_back(expr());
    must_kw("when");
    f = FnKind::CaseWhen;
  }
  for (;;) {
    a.push_back(expr());
    must_kw("then");
    a.push_back(expr());
    int i = must_one_of({"when", "else", "end"});
    if (i == 0) continue;
    if (i == 1) {
      a.push_back(expr());
      must_kw("end");
    } else {
      a.push_back(mk_null());
    }
    break;
  }
  return mk_call(f, sv(), std::move(a));
}

}  // namespace

bool parse(sv sql, Statement &out, ParseError &err) {
  Parser p(sql);
  try {
    p.parse_stmt(out);
    return true;
  } catch (const Fail &) {
    err = std::move(p.err);
    return false;
  }
}

}  // namespace nut::sql
