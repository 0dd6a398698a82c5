// sql_lexer.cpp — see sql_lexer.hpp for the reference map.
#include "sql_lexer.hpp"

namespace nut::sql {

const char *tok_name(Tok t) {
  static const char *names[] = {
      "KeywordOrIdentifier", "DelimitedIdentifier", "ConfigIdentifier", "QueryParameter", "RawStringLiteral",
      "EscapedSingleQuotedStringLiteral", "EscapedDoubleQuotedStringLiteral", "IntegerLiteral", "FloatLiteral",
      "HexLiteral", "Comma", "Dot", "Colon", "SemiColon", "Plus", "Minus", "Mul", "Div", "Mod", "Eq", "NotEq", "Lt",
      "Gt", "LtEq", "GtEq", "LParen", "RParen", "LBracket", "RBracket", "LBrace", "RBrace", "BitAnd", "BitOr",
      "BitXor", "BitNot", "BitLShift", "BitRShift", "Comment", "Whitespace", "EOF"};
  int i = (int)t;
  return (i >= 0 && i <= (int)Tok::Eof) ? names[i] : "?";
}

std::string Position::str() const { return "line " + std::to_string(line) + " col " + std::to_string(col); }

std::string LexError::str() const {
  const char *k = t == LexErr::UnexpectedEOF ? "Unexpected EOF" : t == LexErr::UnexpectedChar ? "Unexpected Char"
                                                                                                 : "Incomplete Token";
  return std::string(k) + ": " + ctx + " near " + pos.str();
}

std::string utf8_encode(int32_t cp) {
  std::string s;
  if (cp < 0x80) {
    s += (char)cp;
  } else if (cp < 0x800) {
    s += (char)(0xC0 | (cp >> 6));
    s += (char)(0x80 | (cp & 0x3F));
  } else if (cp < 0x10000) {
    s += (char)(0xE0 | (cp >> 12));
    s += (char)(0x80 | ((cp >> 6) & 0x3F));
    s += (char)(0x80 | (cp & 0x3F));
  } else {
    s += (char)(0xF0 | (cp >> 18));
    s += (char)(0x80 | ((cp >> 12) & 0x3F));
    s += (char)(0x80 | ((cp >> 6) & 0x3F));
    s += (char)(0x80 | (cp & 0x3F));
  }
  return s;
}

bool valid_utf8(const char *s, size_t n, size_t *bad_at) {
  const unsigned char *u = (const unsigned char *)s;
  size_t i = 0;
  while (i < n) {
    unsigned c = u[i];
    size_t len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    if (len == 0 || i + len > n) {
      if (bad_at) *bad_at = i;
      return false;
    }
    uint32_t cp = len == 1 ? c : len == 2 ? (c & 0x1F) : len == 3 ? (c & 0x0F) : (c & 0x07);
    for (size_t k = 1; k < len; ++k) {
      if ((u[i + k] >> 6) != 2) {
        if (bad_at) *bad_at = i;
        return false;
      }
      cp = (cp << 6) | (u[i + k] & 0x3F);
    }
    // overlong forms, surrogates and out-of-range code points are not valid UTF-8
    if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && cp < 0x10000) || cp > 0x10FFFF ||
        (cp >= 0xD800 && cp <= 0xDFFF)) {
      if (bad_at) *bad_at = i;
      return false;
    }
    i += len;
  }
  return true;
}

int32_t Cursor::peek() {
  if (plen_) return peeked_;
  if (cur_ >= n_) return -1;
  const unsigned char *u = (const unsigned char *)raw_ + cur_;
  unsigned c = u[0];
  if (c < 0x80) {
    plen_ = 1;
    peeked_ = (int32_t)c;
    return peeked_;
  }
  // input validated as UTF-8 by the caller
  int len = (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : 4;
  uint32_t cp = len == 2 ? (c & 0x1F) : len == 3 ? (c & 0x0F) : (c & 0x07);
  for (int k = 1; k < len; ++k) cp = (cp << 6) | (u[k] & 0x3F);
  plen_ = (uint8_t)len;
  peeked_ = (int32_t)cp;
  return peeked_;
}

Position Cursor::pos_at(size_t byte) const {
  Position p;
  size_t i = 0;
  const unsigned char *u = (const unsigned char *)raw_;
  while (i < byte) {
    unsigned c = u[i];
    size_t len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : 4;
    if (c == '\r') {
      if (i + 1 < byte && u[i + 1] == '\n') ++i;
      p.line += 1;
      p.col = 1;
    } else if (c == '\n') {
      p.line += 1;
      p.col = 1;
    } else if (c == '\t') {
      p.col += 4;
    } else {
      p.col += 1;
    }
    i += len;
  }
  return p;
}

namespace {
bool is_ws(int32_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
bool is_digit(int32_t c) { return c >= '0' && c <= '9'; }
bool is_hex(int32_t c) { return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
bool is_ident(int32_t c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_' || is_digit(c); }
bool in(int32_t c, const char *set) {
  for (const char *p = set; *p; ++p)
    if (c == (unsigned char)*p) return true;
  return false;
}
// chars that may follow an identifier / a query parameter / a numeric literal
// (mod.rs:478-543); -1 (end of input) is always fine
bool bad_end_identifier(int32_t c) { return c >= 0 && !in(c, "+-*/%&|^><=!.,;[](){}\t\n\r "); }
bool bad_end_query_param(int32_t c) { return c >= 0 && !in(c, "+-*/%&|^><=!,:;])}\t\n\r "); }
bool bad_end_numeric(int32_t c) { return c >= 0 && !in(c, "+-*/%&|^><=!:,;])}\t\n\r "); }
std::string quoted(int32_t c) { return "'" + utf8_encode(c) + "'"; }
}  // namespace

bool Tokenizer::fail(LexErr t, std::string ctx, LexError &err) {
  err.t = t;
  err.ctx = std::move(ctx);
  err.pos = src_.current_pos();
  return false;
}

bool Tokenizer::next_token(Token &out, LexError &err) {
  src_.pin();
  {
    size_t s = src_.cursor();
    src_.skip_while(is_ws);
    if (s != src_.cursor()) return emit(Tok::Whitespace, out);
  }
  const int32_t c = src_.peek();
  if (c < 0) return emit(Tok::Eof, out);
  auto one = [&](Tok t) {
    src_.consume_peeked();
    return emit(t, out);
  };
  switch (c) {
    case '(': return one(Tok::LParen);
    case ')': return one(Tok::RParen);
    case '[': return one(Tok::LBracket);
    case ']': return one(Tok::RBracket);
    case '{': return one(Tok::LBrace);
    case '}': return one(Tok::RBrace);
    case ',': return one(Tok::Comma);
    case ':': return one(Tok::Colon);
    case '+': return one(Tok::Plus);
    case '*': return one(Tok::Mul);
    case '%': return one(Tok::Mod);
    case '=': return one(Tok::Eq);
    case '&': return one(Tok::BitAnd);
    case '|': return one(Tok::BitOr);
    case '^': return one(Tok::BitXor);
    case '~': return one(Tok::BitNot);
    case ';': return one(Tok::SemiColon);
    case '-': {
      src_.consume_peeked();
      if (src_.peek() == '-') {
        src_.consume_peeked();
        src_.skip_while([](int32_t x) { return x == ' '; });
        Span sp = src_.take_while([](int32_t x) { return x != '\n' && x != '\r'; });
        return emit_on(Tok::Comment, sp, out);
      }
      return emit(Tok::Minus, out);
    }
    case '/': {
      src_.consume_peeked();
      if (src_.peek() == '*') {
        src_.consume_peeked();
        return block_comment_body(out, err);
      }
      return emit(Tok::Div, out);
    }
    case '!': {
      src_.consume_peeked();
      if (src_.peek() == '=') return one(Tok::NotEq);
      return fail(LexErr::UnexpectedChar, "'!' can only be used with '='", err);
    }
    case '<': {
      src_.consume_peeked();
      int32_t n = src_.peek();
      if (n == '=') return one(Tok::LtEq);
      if (n == '>') return one(Tok::NotEq);
      if (n == '<') return one(Tok::BitLShift);
      return emit(Tok::Lt, out);
    }
    case '>': {
      src_.consume_peeked();
      int32_t n = src_.peek();
      if (n == '=') return one(Tok::GtEq);
      if (n == '>') return one(Tok::BitRShift);
      return emit(Tok::Gt, out);
    }
    case '`': return delimited_identifier(out, err);
    case '$': return query_parameter(out, err);
    case '@': return config_identifier(out, err);
    case '\'': return string_literal('\'', Tok::EscapedSQStringLiteral, out, err);
    case '"': return string_literal('"', Tok::EscapedDQStringLiteral, out, err);
    default: break;
  }
  if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_') return keyword_or_identifier(out, err);
  if (c == '.' || is_digit(c)) return dot_or_numeric(out, err);
  return fail(LexErr::UnexpectedChar, quoted(c) + " is invalid outside string literal", err);
}

bool Tokenizer::string_literal(int32_t quote, Tok escaped_kind, Token &out, LexError &err) {
  src_.consume_peeked();  // opening quote
  bool escaped = false;
  src_.pin();             // the span excludes the quotes
  for (;;) {
    int32_t c = src_.peek();
    if (c < 0) return fail(LexErr::UnexpectedEOF, "string literal is not complete", err);
    if (c == quote) {
      Span sp = src_.cut_from_pinned();
      src_.consume_peeked();
      if (src_.peek() == quote) {  // '' -> ' (or "" -> ")
        src_.consume_peeked();
        escaped = true;
      } else {
        return emit_on(escaped ? escaped_kind : Tok::RawStringLiteral, sp, out);
      }
    } else if (c == '\\') {
      src_.consume_peeked();
      int32_t n = src_.next();  // the escaped char, whatever it is
      if (n == '\r' && src_.peek() == '\n') src_.consume_peeked();
      escaped = true;
    } else if (c == '\r') {
      return fail(LexErr::UnexpectedChar, "\\r in string is supported but should be escaped by '\\'", err);
    } else if (c == '\n') {
      return fail(LexErr::UnexpectedChar, "\\n in string is supported but should be escaped by '\\'", err);
    } else {
      src_.consume_peeked();
    }
  }
}

bool Tokenizer::dot_or_numeric(Token &out, LexError &err) {
  src_.pin();
  Span sp = src_.take_while(is_digit);
  if (sp.end - sp.start == 1 && src_.data()[sp.start] == '0') {
    int32_t n = src_.peek();
    if (n == 'x' || n == 'X') {
      src_.consume_peeked();
      Span hx = src_.take_while(is_hex);  // the token excludes "0x"
      return emit_on(Tok::HexLiteral, hx, out);
    }
    if (n != '.') {
      if (bad_end_numeric(n)) return fail(LexErr::UnexpectedChar, quoted(n) + " is invalid in numeric literal", err);
      return emit_on(Tok::IntegerLiteral, sp, out);
    }
  }
  int32_t n = src_.peek();
  if (n == '.') {
    src_.consume_peeked();
  } else {
    if (bad_end_numeric(n)) return fail(LexErr::UnexpectedChar, quoted(n) + " cannot be a part of integer literal", err);
    return emit_on(Tok::IntegerLiteral, sp, out);
  }
  src_.skip_while(is_digit);
  Span all = src_.cut_from_pinned();
  if (all.end - all.start == 1 && src_.data()[all.start] == '.') return emit_on(Tok::Dot, all, out);
  n = src_.peek();
  if (bad_end_numeric(n)) return fail(LexErr::UnexpectedChar, quoted(n) + " cannot be a part of float literal", err);
  return emit_on(Tok::FloatLiteral, all, out);
}

bool Tokenizer::keyword_or_identifier(Token &out, LexError &err) {
  Span sp = src_.take_while(is_ident);
  int32_t n = src_.peek();
  if (bad_end_identifier(n))
    return fail(LexErr::UnexpectedChar, quoted(n) + " cannot be a part of identifier or keyword", err);
  return emit_on(Tok::KeywordOrIdentifier, sp, out);
}

bool Tokenizer::config_identifier(Token &out, LexError &err) {
  src_.consume_peeked();  // '@'
  if (is_digit(src_.peek()))
    return fail(LexErr::UnexpectedChar, "config identifier cannot starts with numbers", err);
  Span sp = src_.take_while(is_ident);
  int32_t n = src_.peek();
  if (bad_end_identifier(n))
    return fail(LexErr::UnexpectedChar, quoted(n) + " cannot be a part of config identifier", err);
  if (sp.empty()) return fail(LexErr::Incomplete, "identifier should have name", err);
  return emit_on(Tok::ConfigIdentifier, sp, out);
}

bool Tokenizer::delimited_identifier(Token &out, LexError &err) {
  src_.consume_peeked();  // '`'
  Span sp = src_.take_while([](int32_t x) { return x != '`' && x != '\r' && x != '\n'; });
  if (sp.empty()) return fail(LexErr::Incomplete, "delimited identifier cannot be an empty string", err);
  int32_t n = src_.peek();
  if (n == '`') {
    src_.consume_peeked();
    return emit_on(Tok::DelimitedIdentifier, sp, out);
  }
  if (n >= 0)
    return fail(LexErr::UnexpectedChar, "'\\r' or '\\n' cannot be a part of delimited identifier", err);
  return fail(LexErr::UnexpectedEOF, "delimited identifier is not complete", err);
}

bool Tokenizer::query_parameter(Token &out, LexError &err) {
  src_.consume_peeked();  // '$'
  Span sp = src_.take_while(is_digit);
  int32_t n = src_.peek();
  if (bad_end_query_param(n))
    return fail(LexErr::UnexpectedChar, quoted(n) + " cannot be a part of query parameter", err);
  if (sp.empty()) return fail(LexErr::Incomplete, "query parameter should have an index", err);
  return emit_on(Tok::QueryParameter, sp, out);
}

bool Tokenizer::block_comment_body(Token &out, LexError &err) {
  size_t start = src_.cursor(), end = src_.cursor();
  int state = 0;  // 0 in comment, 1 after '*', 2 closed
  while (state != 2) {
    int32_t c = src_.peek();
    if (c < 0) return fail(LexErr::UnexpectedEOF, "block comment is not complete", err);
    src_.consume_peeked();
    if (state == 1 && c == '/')
      state = 2;
    else
      state = c == '*' ? 1 : 0;
    if (state == 0) end = src_.cursor();
  }
  return emit_on(Tok::Comment, Span{start, end}, out);
}

}  // namespace nut::sql
