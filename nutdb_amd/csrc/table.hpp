// table.hpp — typed device tables from CREATE TABLE.
//
// Not a storage engine: a table is a set of HBM-resident columns in the executed
// representation (int64 / f64) plus, for string-like columns, a host dictionary.
//   declared type (ast/item.rs:14-68)           HBM column
//   Int8..Int64, UInt8..UInt32, Serial*, UInt64  int64 (sign/zero-extended on the GPU;
//                                                 UInt64 values >= 2^63 are rejected)
//   Boolean                                      int64 0/1
//   Date / Datetime                              int64 days / seconds since 1970-01-01
//   Float32 / Float64                            f64 (Float32 widened exactly)
//   String / Chars(n) / Dictionary(String)       int64 codes into the table's dictionary
//   Enum('a' = 1, ...)                           int64 declared ids
//   Nullable(T)                                  T (a NULL value is rejected at load)
// Codes of one table share one dictionary, so string columns compare with each other;
// codes are in first-seen order (no ordering), so strings support = / != / IN only.
#pragma once

#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.hpp"

namespace nut {

struct Dict {
  std::vector<std::string> strs;                 // code -> string (an overlay: codes from base_n on)
  std::unordered_map<std::string, int64_t> codes;  // string -> code
  bool fixed = false;                            // Enum: the declaration is the dictionary
  // A query-local overlay over a table's dictionary: strings a query derives
  // (substring results) get codes after the base's, in the overlay only — the table's
  // dictionary is never written during a query, so concurrent queries only read it and no
  // query's strings leak into another's per-code tables.
  const Dict *base = nullptr;
  size_t base_n = 0;
  static Dict overlay(const Dict *b) {
    Dict o;
    o.base = b;
    o.base_n = b->strs.size();
    return o;
  }
  size_t size() const { return base_n + strs.size(); }  // codes [0, size()) (not Enum)
  const std::string &at(size_t c) const { return c < base_n ? base->strs[c] : strs[c - base_n]; }
  int64_t find(const std::string &s) const {
    if (base) {
      const int64_t b = base->find(s);
      if (b >= 0) return b;
    }
    auto it = codes.find(s);
    return it == codes.end() ? -1 : it->second;
  }
  // the code of s, appended to this dictionary if absent (overlays and table loads only)
  int64_t intern(std::string s) {
    const int64_t k = find(s);
    if (k >= 0) return k;
    const int64_t code = (int64_t)size();
    codes.emplace(s, code);
    strs.push_back(std::move(s));
    return code;
  }
  const std::string *decode(int64_t c) const {
    if (fixed) {
      for (const auto &kv : codes)
        if (kv.second == c) return &kv.first;
      return nullptr;
    }
    return c >= 0 && (uint64_t)c < size() ? &at((size_t)c) : nullptr;
  }
};

// the overlays of one execution: one per table dictionary it binds (Enums stay as they are)
struct DictOverlays {
  std::vector<std::pair<const Dict *, std::unique_ptr<Dict>>> o;
  const Dict *of(const Dict *d) {
    if (!d || d->fixed) return d;
    for (auto &x : o)
      if (x.first == d) return x.second.get();
    o.emplace_back(d, std::unique_ptr<Dict>(new Dict(Dict::overlay(d))));
    return o.back().second.get();
  }
};

struct TCol {
  std::string name;
  int kind = NUT_COL_INT;  // nut_col_kind
  int width = 8;           // bytes of one appended host value (numeric kinds)
  int exec_type = NUT_T_I64;
  Dict *dict = nullptr;    // STRING: the table's shared dictionary; ENUM: own
  Dict own;                // ENUM
  void *dev = nullptr;     // HBM column, 8 B per row
  uint64_t n = 0, cap = 0;
};

}  // namespace nut

struct nut_table {
  std::string name;
  std::vector<nut::TCol> cols;
  nut::Dict strings;  // shared by every string-like column
  int device = -1;    // device of the columns (set by the first append)
  uint64_t rows() const {
    if (cols.empty()) return 0;
    uint64_t n = cols[0].n;
    for (const auto &c : cols) n = c.n < n ? c.n : n;
    return n;
  }
  bool ragged() const {
    for (const auto &c : cols)
      if (c.n != cols[0].n) return true;
    return false;
  }
};
