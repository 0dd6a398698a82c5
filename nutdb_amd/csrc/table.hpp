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

#include <string>
#include <unordered_map>
#include <vector>

#include "common.hpp"

namespace nut {

struct Dict {
  std::vector<std::string> strs;                 // code -> string
  std::unordered_map<std::string, int64_t> codes;  // string -> code
  bool fixed = false;                            // Enum: the declaration is the dictionary
  int64_t find(const std::string &s) const {
    auto it = codes.find(s);
    return it == codes.end() ? -1 : it->second;
  }
  const std::string *decode(int64_t c) const {
    if (fixed) {
      for (const auto &kv : codes)
        if (kv.second == c) return &kv.first;
      return nullptr;
    }
    return c >= 0 && (uint64_t)c < strs.size() ? &strs[(size_t)c] : nullptr;
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
