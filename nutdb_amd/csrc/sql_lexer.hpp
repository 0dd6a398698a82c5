// sql_lexer.hpp — tokenizer of the NutDB SQL dialect (C++ restatement of the reference
// front end).
//
// Follows /root/reference/src/parser/tokenizer/:
//   token kinds .......... token.rs:5-91 (40 kinds; whitespace and comments are tokens)
//   next_token ........... mod.rs:66-112
//   strings .............. mod.rs:115-184 ('' / "" doubling, backslash escapes, raw CR/LF
//                          is an error, RawStringLiteral when nothing was escaped)
//   numerics ............. mod.rs:191-260 (0x hex, ".5" and "1." floats, a lone "." is Dot,
//                          a char that cannot end a numeric is an error)
//   identifiers .......... mod.rs:262-345 (ASCII [A-Za-z_][A-Za-z0-9_]*, `delimited`, @config)
//   $n parameters ........ mod.rs:347-365;  comments mod.rs:367-468
//   positions ............ utf8_iter.rs:89-116 (line/col by chars; '\t' = 4 cols; "\r\n"
//                          is one line break)
// Spans are byte offsets into the input, which must be valid UTF-8.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>

namespace nut::sql {

enum class Tok : int32_t {
  KeywordOrIdentifier = 0,
  DelimitedIdentifier,
  ConfigIdentifier,
  QueryParameter,
  RawStringLiteral,
  EscapedSQStringLiteral,
  EscapedDQStringLiteral,
  IntegerLiteral,
  FloatLiteral,
  HexLiteral,
  Comma,
  Dot,
  Colon,
  SemiColon,
  Plus,
  Minus,
  Mul,
  Div,
  Mod,
  Eq,
  NotEq,
  Lt,
  Gt,
  LtEq,
  GtEq,
  LParen,
  RParen,
  LBracket,
  RBracket,
  LBrace,
  RBrace,
  BitAnd,
  BitOr,
  BitXor,
  BitNot,
  BitLShift,
  BitRShift,
  Comment,
  Whitespace,
  Eof,
};

// Display names (derive_more Display of TokenType, token.rs:5-91)
const char *tok_name(Tok t);

struct Span {
  size_t start = 0, end = 0;
  bool empty() const { return start == end; }
};

struct Token {
  Tok t = Tok::Eof;
  Span span;
  bool is_whitespace() const { return t == Tok::Whitespace || t == Tok::Comment; }
  bool maybe_keyword() const { return t == Tok::KeywordOrIdentifier; }
  bool is_terminator() const { return t == Tok::Eof || t == Tok::SemiColon; }
};

struct Position {
  size_t line = 1, col = 1;
  std::string str() const;  // "line L col C"
};

enum class LexErr { UnexpectedEOF, UnexpectedChar, Incomplete };

struct LexError {
  LexErr t;
  std::string ctx;
  Position pos;
  std::string str() const;  // "{kind}: {ctx} near {pos}"
};

// Decoding cursor over UTF-8 with a one-char peek buffer (utf8_iter.rs:40-237).
class Cursor {
 public:
  Cursor(const char *s, size_t n) : raw_(s), n_(n) {}
  size_t cursor() const { return cur_; }
  void pin() { pinned_ = cur_; }
  Span cut_from_pinned() const { return Span{pinned_, cur_}; }
  std::string slice(const Span &s) const { return std::string(raw_ + s.start, s.end - s.start); }
  const char *data() const { return raw_; }
  size_t size() const { return n_; }
  // code point of the next char, or -1 at end
  int32_t peek();
  int32_t next() {
    int32_t c = peek();
    consume_peeked();
    return c;
  }
  void consume_peeked() {
    cur_ += plen_;
    plen_ = 0;
  }
  template <class P>
  Span take_while(P pred) {
    size_t s = cur_;
    skip_while(pred);
    return Span{s, cur_};
  }
  template <class P>
  void skip_while(P pred) {
    for (;;) {
      int32_t c = peek();
      if (c >= 0 && pred(c)) {
        consume_peeked();
        continue;
      }
      break;
    }
  }
  Position pos_at(size_t byte) const;
  Position current_pos() const { return pos_at(cur_); }

 private:
  const char *raw_;
  size_t n_;
  size_t cur_ = 0, pinned_ = 0;
  int32_t peeked_ = 0;
  uint8_t plen_ = 0;
};

class Tokenizer {
 public:
  Tokenizer(const char *s, size_t n) : src_(s, n) {}
  // false on a lexical error (err filled)
  bool next_token(Token &out, LexError &err);
  const Cursor &source() const { return src_; }

 private:
  Cursor src_;
  bool fail(LexErr t, std::string ctx, LexError &err);
  bool emit(Tok t, Token &out) {
    out.t = t;
    out.span = src_.cut_from_pinned();
    return true;
  }
  bool emit_on(Tok t, Span s, Token &out) {
    out.t = t;
    out.span = s;
    return true;
  }
  bool string_literal(int32_t quote, Tok escaped_kind, Token &out, LexError &err);
  bool dot_or_numeric(Token &out, LexError &err);
  bool keyword_or_identifier(Token &out, LexError &err);
  bool config_identifier(Token &out, LexError &err);
  bool delimited_identifier(Token &out, LexError &err);
  bool query_parameter(Token &out, LexError &err);
  bool block_comment_body(Token &out, LexError &err);
};

// true if `input` is valid UTF-8 (the reference takes &str, which guarantees it)
bool valid_utf8(const char *s, size_t n, size_t *bad_at);
std::string utf8_encode(int32_t cp);

}  // namespace nut::sql
