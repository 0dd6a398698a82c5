// sql_ast.hpp — statement tree produced by the SQL front end.
//
// Restates the reference AST (/root/reference/src/parser/ast/):
//   Statement + statement payloads ....... ast/mod.rs:13-107
//   Expr / UnaryOp / BinaryOp / FnCall .... ast/expr.rs:7-41
//   Literal, Identifier, data types, ops .. ast/item.rs:8-228
//   Query / QueryBody / clauses ........... ast/query.rs:21-173
//   Alter actions ......................... ast/alter.rs:7-58
// Identifiers and raw string literals are views into the statement's own copy of
// the SQL text (the reference borrows the caller's &str the same way); unescaped
// strings are owned (the reference's Cow::Owned).
#pragma once

#include <stdint.h>

#include <memory>
#include <optional>
#include <string>
#include <string_view>
#include <vector>

namespace nut::sql {

using sv = std::string_view;
typedef unsigned __int128 u128;

struct Query;

// ------------------------------------------------------------------ literals
enum class IntervalUnit : uint8_t { Second, Minute, Hour, Day, Month, Year };

// Exact decimal (bigdecimal 0.3 BigDecimal): value = (neg ? -1 : 1) * digits * 10^-scale.
// `digits` is the decimal digit string of the integer mantissa without leading zeros
// ("" is zero).  Equality is numeric (BigDecimal's PartialEq aligns scales).
struct Decimal {
  bool neg = false;
  std::string digits;
  int64_t scale = 0;
  bool is_zero() const { return digits.empty(); }
  std::string str() const;   // BigDecimal Display: the scale is kept ("0.0001000000")
  double to_f64() const;     // correctly rounded
  bool operator==(const Decimal &o) const;
};

enum class LitKind : uint8_t { Integer, Float, String, Boolean, Interval, Null };

struct Literal {
  LitKind k = LitKind::Null;
  u128 mag = 0;          // Integer magnitude (item.rs:91: Integer(u128, positive))
  bool positive = true;  // Integer sign; Boolean value
  Decimal dec;           // Float
  std::string str;       // String (unescaped)
  uint64_t interval = 0; // Interval count
  IntervalUnit unit = IntervalUnit::Day;
  // derive(PartialEq) on Literal (item.rs:89): structural, so Integer(1) != Float(1.0)
  // and Integer(0,false) != Integer(0,true)
  bool operator==(const Literal &o) const;
};

// ------------------------------------------------------------------ expressions
enum class UnOp : uint8_t { BitwiseNot, Not, IsNull, IsNotNull };
enum class BinOp : uint8_t {
  Plus, Minus, Multi, Div, Mod, Gt, Lt, GtEq, LtEq, Eq, NotEq, And, Or, Xor, Like, NotLike,
  ILike, NotILike, In, NotIn, IndexAccess, BitwiseOr, BitwiseAnd, BitwiseXor,
  BitwiseLeftShift, BitwiseRightShift,
};
enum class FnKind : uint8_t { If, MultiIf, CaseWhen, Between, NotBetween, Exists, NotExists, Others };
enum class CollType : uint8_t { Tuple, Map, Array };
enum class EK : uint8_t { Identifier, QueryParameter, Literal, Collection, UnaryOp, BinaryOp, FnCall, Subquery };

struct Identifier {
  bool wildcard = false;
  sv name;               // Word(name) unless wildcard
  bool qualified = false;
  sv qualifier;
};

struct Expr {
  EK k = EK::Literal;
  uint8_t op = 0;                 // UnOp / BinOp / CollType / FnKind
  Identifier id;                  // Identifier; FnCall Others(name) keeps the name in id.name
  uint64_t param = 0;             // QueryParameter index
  std::unique_ptr<Literal> lit;   // Literal
  std::vector<Expr> kids;         // operand(s), collection items, call arguments
  std::unique_ptr<Query> q;       // Subquery

  Expr();
  Expr(Expr &&) noexcept;
  Expr &operator=(Expr &&) noexcept;
  ~Expr();

  bool is_lit() const { return k == EK::Literal; }
  bool is_bool_lit(bool *b) const {
    if (k == EK::Literal && lit->k == LitKind::Boolean) {
      *b = lit->positive;
      return true;
    }
    return false;
  }
  UnOp uop() const { return (UnOp)op; }
  BinOp bop() const { return (BinOp)op; }
  FnKind fn() const { return (FnKind)op; }
};

// ------------------------------------------------------------------ queries
struct QueryExpr {
  Expr e;
  std::optional<sv> alias;
};

enum class SourceKind : uint8_t { TableFn, Table, Subquery };
struct QuerySource {
  SourceKind k = SourceKind::Table;
  sv table;   // Table
  Expr e;     // TableFn (an FnCall expr) or Subquery (a Subquery expr)
  std::optional<sv> alias;
};

enum class JoinType : uint8_t { Inner, FullOuter, LeftOuter, RightOuter, LeftSemi, RightSemi, LeftAnti, RightAnti, AsOf };
struct JoinClause {
  JoinType t = JoinType::Inner;
  QuerySource src;
  bool on = true;
  Expr cond;                        // On
  std::vector<Identifier> using_;   // Using
};

struct OrderKey {
  QueryExpr e;
  bool desc = false;
};

struct LimitClause {
  uint64_t size = 0, offset = 0;
  bool with_ties = false;
};

struct CTE {
  std::unique_ptr<Query> q;
  sv alias;
};

struct QueryBody {
  std::optional<std::vector<CTE>> with;
  bool distinct = false;
  std::optional<std::vector<QueryExpr>> distinct_on;
  std::vector<QueryExpr> columns;
  std::optional<QuerySource> from;
  std::vector<JoinClause> joins;
  std::optional<Expr> where;
  std::optional<std::vector<QueryExpr>> group_by;
  std::optional<Expr> having;
  std::optional<std::vector<OrderKey>> order_by;
  std::optional<LimitClause> limit;
};

enum class UnionType : uint8_t { UnionAll, UnionDistinct, Intersect, Except };
struct Query {
  bool is_union = false;
  std::unique_ptr<QueryBody> body;   // Single
  UnionType ut = UnionType::UnionAll;
  std::unique_ptr<Query> l, r;       // Union
};

// ------------------------------------------------------------------ DDL pieces
enum class Scalar : uint8_t {
  Int8, Int16, Int32, Int64, Int128, UInt8, UInt16, UInt32, UInt64, UInt128, Serial32, Serial64,
  Serial128, USerial32, USerial64, USerial128, Decimal32, Decimal64, Float32, Float64, Boolean,
  Chars, String, Uuid, Date, Datetime,
};
enum class Compound : uint8_t { Array, Enum, Tuple, Map, Dictionary, Nullable };

struct EnumBind {
  uint64_t id = 0;
  std::string literal;
};

struct DataType {
  bool scalar = true;
  Scalar s = Scalar::Int64;
  uint64_t param = 0;            // Decimal scale, Chars length, String max_length
  Compound c = Compound::Array;
  std::vector<DataType> kids;    // Array/Dictionary/Nullable: 1; Tuple: n; Map: (value, key)
  std::vector<EnumBind> binds;   // Enum
};

struct ColumnDef {
  sv name;
  DataType t;
  std::optional<Expr> default_;
  std::optional<std::string> comment;
};
struct ConstraintDef {
  sv name;
  Expr check;
};
struct IndexDef {
  sv name;
  Expr indexer;   // an FnCall expr
};

struct TableDef {
  sv name;
  std::vector<ColumnDef> columns;
  std::vector<ConstraintDef> constraints;
  std::vector<IndexDef> indexes;
  std::optional<std::vector<Expr>> primary_key, order_by;
  std::optional<Expr> partition_by;
  std::optional<std::string> comment;
};

struct ViewDef {
  sv name, strategy;
  std::optional<std::vector<Expr>> primary_key, order_by;
  std::optional<Expr> partition_by;
  Query query;
  std::optional<std::string> comment;
};

// ------------------------------------------------------------------ statements
enum class StmtKind : uint8_t { Select, Insert, Explain, Alter, Create, Describe, Drop, Truncate, Optimize, Set };

enum class InsertKind : uint8_t { Rows, Subquery, FnCall };
struct InsertStmt {
  sv table;
  std::optional<std::vector<sv>> columns;
  InsertKind k = InsertKind::Rows;
  uint64_t column_size = 0;
  std::vector<Expr> data;   // Rows, row-major
  Query query;              // Subquery
  Expr fn;                  // FnCall
};

enum class AlterKind : uint8_t { Add, Rename, Drop };
enum class EntityKind : uint8_t { Column, Constraint, Index, Partition, Table };
enum class Position_ : uint8_t { First, After, Last };
struct AlterStmt {
  sv table;
  AlterKind k = AlterKind::Add;
  EntityKind entity = EntityKind::Column;
  bool if_flag = false;         // Add: if_not_exists; Drop: if_exists
  ColumnDef column;             // Add Column
  ConstraintDef constraint;     // Add Constraint
  IndexDef index;               // Add Index
  Position_ pos = Position_::Last;
  sv after;                     // Add ... AFTER name
  sv name;                      // Rename/Drop entity name
  std::string partition;        // Drop Partition '<literal>'
  sv new_name;                  // Rename
};

enum class DescribeKind : uint8_t { Database, Table, View };

struct Statement {
  StmtKind k = StmtKind::Select;
  Query query;                                 // Select / Explain
  std::unique_ptr<InsertStmt> insert;
  std::unique_ptr<AlterStmt> alter;
  bool if_flag = false;                        // Create: if_not_exists; Drop/Truncate: if_exists
  bool is_view = false;                        // Create/Drop/Truncate entity; Describe View
  std::unique_ptr<TableDef> table;             // Create Table
  std::unique_ptr<ViewDef> view;               // Create View
  DescribeKind describe = DescribeKind::Database;
  sv name;                                     // Describe/Drop/Truncate/Optimize/Set name
  std::optional<Expr> value;                   // Optimize partition / Set value
};

// ------------------------------------------------------------------ front end
struct ParseError {
  bool lex = false;   // LexError vs SyntaxError (error.rs:8-14)
  std::string msg;    // Display text of the inner error
  std::string str() const { return (lex ? "Lex Error: " : "Syntax Error: ") + msg; }
};

// Parser::parse (mod.rs:26-29).  `sql` must stay alive as long as `out`.
bool parse(sv sql, Statement &out, ParseError &err);

// literal.rs:36-103 (throws nothing; false + err on an invalid \u{...} escape)
bool unescape(sv raw, char quote, std::string &out, ParseError &err);

// S-expression rendering of a statement (for tests and tools; DESIGN.md §front end)
std::string dump(const Statement &s);
std::string dump(const Expr &e);

}  // namespace nut::sql
