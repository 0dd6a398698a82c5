// sql_dump.cpp — S-expression rendering of the statement tree (sql_ast.hpp).
//
// The reference has no printer beyond #[derive(Debug)]; this compact form exists so
// tests can pin tree SHAPE (precedence, folding, quirks) and tools can inspect what the
// planner lowers from.  Grammar (one node per parenthesised form):
//   literals    (int 5) (int -5) (float 0.50) (str "a\"b") (bool true) null (interval 90 day)
//   identifiers (id name) (id q.name) (id *) (id q.*)      names outside [A-Za-z0-9_] in `...`
//   operators   (+ a b) (<= a b) (and a b) (not-in a b) (index a b) (not a) (is-null a) ...
//   calls       (call name args...) (if ..) (multi-if ..) (case-when ..) (between ..) (exists ..)
//   queries     (body (columns ..) (from ..) (join ..) (where ..) (group-by ..) (having ..)
//                     (order-by (asc e) (desc e)) (limit size offset [ties])) | (union-all L R) ...
#include <stdio.h>

#include "sql_ast.hpp"

namespace nut::sql {
namespace {

const char *kBin[] = {"+",  "-",  "*",   "/",   "%",        ">",  "<",       ">=",       "<=",
                      "=",  "!=", "and", "or",  "xor",      "like", "not-like", "ilike", "not-ilike",
                      "in", "not-in", "index", "|", "&", "^", "<<", ">>"};
const char *kUn[] = {"bitnot", "not", "is-null", "is-not-null"};
const char *kFn[] = {"if", "multi-if", "case-when", "between", "not-between", "exists", "not-exists", "call"};
const char *kColl[] = {"tuple", "map", "array"};
const char *kUnit[] = {"second", "minute", "hour", "day", "month", "year"};
const char *kJoin[] = {"inner", "full-outer", "left-outer", "right-outer", "left-semi",
                       "right-semi", "left-anti", "right-anti", "asof"};
const char *kUnion[] = {"union-all", "union-distinct", "intersect", "except"};
const char *kScalar[] = {"Int8",      "Int16",     "Int32",      "Int64",    "Int128",    "UInt8",   "UInt16",
                         "UInt32",    "UInt64",    "UInt128",    "Serial32", "Serial64",  "Serial128",
                         "USerial32", "USerial64", "USerial128", "Decimal32", "Decimal64", "Float32", "Float64",
                         "Boolean",   "Chars",     "String",     "Uuid",     "Date",      "Datetime"};
const char *kCompound[] = {"Array", "Enum", "Tuple", "Map", "Dictionary", "Nullable"};

std::string u128_str(u128 v) {
  if (v == 0) return "0";
  char buf[48];
  int i = 47;
  buf[i] = 0;
  while (v) {
    buf[--i] = (char)('0' + (int)(v % 10));
    v /= 10;
  }
  return std::string(buf + i);
}

void quote(std::string &o, sv s) {
  o += '"';
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += (char)c;
    } else if (c == '\n') {
      o += "\\n";
    } else if (c == '\r') {
      o += "\\r";
    } else if (c == '\t') {
      o += "\\t";
    } else if (c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\x%02x", c);
      o += b;
    } else {
      o += (char)c;
    }
  }
  o += '"';
}

void name(std::string &o, sv s) {
  bool plain = !s.empty();
  for (unsigned char c : s)
    if (!((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_')) plain = false;
  if (plain) {
    o += s;
  } else {
    o += '`';
    o += s;
    o += '`';
  }
}

struct D {
  std::string o;

  void lit(const Literal &l) {
    switch (l.k) {
      case LitKind::Integer:
        o += "(int ";
        if (!l.positive) o += '-';
        o += u128_str(l.mag);
        o += ')';
        break;
      case LitKind::Float: o += "(float " + l.dec.str() + ")"; break;
      case LitKind::String:
        o += "(str ";
        quote(o, l.str);
        o += ')';
        break;
      case LitKind::Boolean: o += l.positive ? "(bool true)" : "(bool false)"; break;
      case LitKind::Interval:
        o += "(interval " + std::to_string(l.interval) + " " + kUnit[(int)l.unit] + ")";
        break;
      case LitKind::Null: o += "null"; break;
    }
  }

  void ident(const Identifier &id) {
    o += "(id ";
    if (id.qualified) {
      name(o, id.qualifier);
      o += '.';
    }
    if (id.wildcard)
      o += '*';
    else
      name(o, id.name);
    o += ')';
  }

  void kids(const std::vector<Expr> &v) {
    for (const Expr &e : v) {
      o += ' ';
      expr(e);
    }
  }

  void expr(const Expr &e) {
    switch (e.k) {
      case EK::Identifier: ident(e.id); break;
      case EK::QueryParameter: o += "(param " + std::to_string(e.param) + ")"; break;
      case EK::Literal: lit(*e.lit); break;
      case EK::Collection:
        o += '(';
        o += kColl[e.op];
        kids(e.kids);
        o += ')';
        break;
      case EK::UnaryOp:
        o += '(';
        o += kUn[e.op];
        kids(e.kids);
        o += ')';
        break;
      case EK::BinaryOp:
        o += '(';
        o += kBin[e.op];
        kids(e.kids);
        o += ')';
        break;
      case EK::FnCall:
        o += '(';
        o += kFn[e.op];
        if (e.fn() == FnKind::Others) {
          o += ' ';
          name(o, e.id.name);
        }
        kids(e.kids);
        o += ')';
        break;
      case EK::Subquery:
        o += "(subquery ";
        query(*e.q);
        o += ')';
        break;
    }
  }

  void qexpr(const QueryExpr &q) {
    if (q.alias) {
      o += "(as ";
      expr(q.e);
      o += ' ';
      name(o, *q.alias);
      o += ')';
    } else {
      expr(q.e);
    }
  }

  void qexprs(const char *tag, const std::vector<QueryExpr> &v) {
    o += '(';
    o += tag;
    for (const QueryExpr &q : v) {
      o += ' ';
      qexpr(q);
    }
    o += ')';
  }

  void exprs(const char *tag, const std::vector<Expr> &v) {
    o += '(';
    o += tag;
    kids(v);
    o += ')';
  }

  void source(const QuerySource &s) {
    if (s.alias) o += "(as ";
    switch (s.k) {
      case SourceKind::Table:
        o += "(table ";
        name(o, s.table);
        o += ')';
        break;
      case SourceKind::TableFn:
        o += "(table-fn ";
        expr(s.e);
        o += ')';
        break;
      case SourceKind::Subquery: expr(s.e); break;
    }
    if (s.alias) {
      o += ' ';
      name(o, *s.alias);
      o += ')';
    }
  }

  void body(const QueryBody &b) {
    o += "(body";
    if (b.with) {
      o += " (with";
      for (const CTE &c : *b.with) {
        o += " (cte ";
        name(o, c.alias);
        o += ' ';
        query(*c.q);
        o += ')';
      }
      o += ')';
    }
    if (b.distinct) {
      o += " (distinct";
      if (b.distinct_on) {
        o += ' ';
        qexprs("on", *b.distinct_on);
      }
      o += ')';
    }
    o += ' ';
    qexprs("columns", b.columns);
    if (b.from) {
      o += " (from ";
      source(*b.from);
      o += ')';
    }
    for (const JoinClause &j : b.joins) {
      o += " (join ";
      o += kJoin[(int)j.t];
      o += ' ';
      source(j.src);
      if (j.on) {
        o += " (on ";
        expr(j.cond);
        o += ')';
      } else {
        o += " (using";
        for (const Identifier &id : j.using_) {
          o += ' ';
          ident(id);
        }
        o += ')';
      }
      o += ')';
    }
    if (b.where) {
      o += " (where ";
      expr(*b.where);
      o += ')';
    }
    if (b.group_by) {
      o += ' ';
      qexprs("group-by", *b.group_by);
    }
    if (b.having) {
      o += " (having ";
      expr(*b.having);
      o += ')';
    }
    if (b.order_by) {
      o += " (order-by";
      for (const OrderKey &k : *b.order_by) {
        o += k.desc ? " (desc " : " (asc ";
        qexpr(k.e);
        o += ')';
      }
      o += ')';
    }
    if (b.limit) {
      o += " (limit " + std::to_string(b.limit->size) + " " + std::to_string(b.limit->offset);
      if (b.limit->with_ties) o += " ties";
      o += ')';
    }
    o += ')';
  }

  void query(const Query &q) {
    if (!q.is_union) {
      body(*q.body);
      return;
    }
    o += '(';
    o += kUnion[(int)q.ut];
    o += ' ';
    query(*q.l);
    o += ' ';
    query(*q.r);
    o += ')';
  }

  void type(const DataType &t) {
    if (t.scalar) {
      bool param = t.s == Scalar::Decimal32 || t.s == Scalar::Decimal64 || t.s == Scalar::Chars ||
                   t.s == Scalar::String;
      if (param) o += '(';
      o += kScalar[(int)t.s];
      if (param) o += " " + std::to_string(t.param) + ")";
      return;
    }
    o += '(';
    o += kCompound[(int)t.c];
    if (t.c == Compound::Enum) {
      for (const EnumBind &b : t.binds) {
        o += " (";
        quote(o, b.literal);
        o += " " + std::to_string(b.id) + ")";
      }
    }
    for (const DataType &k : t.kids) {
      o += ' ';
      type(k);
    }
    o += ')';
  }

  void column(const ColumnDef &c) {
    o += "(column ";
    name(o, c.name);
    o += ' ';
    type(c.t);
    if (c.default_) {
      o += " (default ";
      expr(*c.default_);
      o += ')';
    }
    if (c.comment) {
      o += " (comment ";
      quote(o, *c.comment);
      o += ')';
    }
    o += ')';
  }

  void constraint(const ConstraintDef &c) {
    o += "(constraint ";
    name(o, c.name);
    o += ' ';
    expr(c.check);
    o += ')';
  }

  void index(const IndexDef &d) {
    o += "(index ";
    name(o, d.name);
    o += ' ';
    expr(d.indexer);
    o += ')';
  }

  void attrs(const std::optional<std::vector<Expr>> &pk, const std::optional<std::vector<Expr>> &ob,
             const std::optional<Expr> &pb, const std::optional<std::string> &cm) {
    if (pk) {
      o += ' ';
      exprs("primary-key", *pk);
    }
    if (ob) {
      o += ' ';
      exprs("order-by", *ob);
    }
    if (pb) {
      o += " (partition-by ";
      expr(*pb);
      o += ')';
    }
    if (cm) {
      o += " (comment ";
      quote(o, *cm);
      o += ')';
    }
  }

  void stmt(const Statement &s) {
    switch (s.k) {
      case StmtKind::Select:
        o += "(select ";
        query(s.query);
        o += ')';
        break;
      case StmtKind::Explain:
        o += "(explain ";
        query(s.query);
        o += ')';
        break;
      case StmtKind::Insert: {
        const InsertStmt &i = *s.insert;
        o += "(insert ";
        name(o, i.table);
        if (i.columns) {
          o += " (columns";
          for (sv c : *i.columns) {
            o += ' ';
            name(o, c);
          }
          o += ')';
        }
        if (i.k == InsertKind::Rows) {
          o += " (rows " + std::to_string(i.column_size);
          kids(i.data);
          o += ')';
        } else if (i.k == InsertKind::Subquery) {
          o += " (query ";
          query(i.query);
          o += ')';
        } else {
          o += " (fn ";
          expr(i.fn);
          o += ')';
        }
        o += ')';
        break;
      }
      case StmtKind::Create:
        o += "(create";
        if (s.if_flag) o += " if-not-exists";
        if (!s.is_view) {
          const TableDef &t = *s.table;
          o += " (table ";
          name(o, t.name);
          o += " (columns";
          for (const ColumnDef &c : t.columns) {
            o += ' ';
            column(c);
          }
          o += ") (constraints";
          for (const ConstraintDef &c : t.constraints) {
            o += ' ';
            constraint(c);
          }
          o += ") (indexes";
          for (const IndexDef &d : t.indexes) {
            o += ' ';
            index(d);
          }
          o += ')';
          attrs(t.primary_key, t.order_by, t.partition_by, t.comment);
          o += ')';
        } else {
          const ViewDef &v = *s.view;
          o += " (view ";
          name(o, v.name);
          o += " (update-by ";
          name(o, v.strategy);
          o += ')';
          attrs(v.primary_key, v.order_by, v.partition_by, v.comment);
          o += ' ';
          query(v.query);
          o += ')';
        }
        o += ')';
        break;
      case StmtKind::Alter: {
        const AlterStmt &a = *s.alter;
        static const char *ent[] = {"column", "constraint", "index", "partition", "table"};
        o += "(alter ";
        name(o, a.table);
        if (a.k == AlterKind::Add) {
          o += " (add";
          if (a.if_flag) o += " if-not-exists";
          o += ' ';
          if (a.entity == EntityKind::Column)
            column(a.column);
          else if (a.entity == EntityKind::Index)
            index(a.index);
          else
            constraint(a.constraint);
          if (a.pos == Position_::First) o += " first";
          if (a.pos == Position_::After) {
            o += " (after ";
            name(o, a.after);
            o += ')';
          }
          o += ')';
        } else if (a.k == AlterKind::Drop) {
          o += " (drop";
          if (a.if_flag) o += " if-exists";
          o += ' ';
          o += ent[(int)a.entity];
          o += ' ';
          if (a.entity == EntityKind::Partition)
            quote(o, a.partition);
          else
            name(o, a.name);
          o += ')';
        } else {
          o += " (rename ";
          o += ent[(int)a.entity];
          if (a.entity != EntityKind::Table) {
            o += ' ';
            name(o, a.name);
          }
          o += ' ';
          name(o, a.new_name);
          o += ')';
        }
        o += ')';
        break;
      }
      case StmtKind::Describe:
        if (s.describe == DescribeKind::Database) {
          o += "(describe database)";
        } else {
          o += s.describe == DescribeKind::Table ? "(describe table " : "(describe view ";
          name(o, s.name);
          o += ')';
        }
        break;
      case StmtKind::Drop:
      case StmtKind::Truncate:
        o += s.k == StmtKind::Drop ? "(drop " : "(truncate ";
        o += s.is_view ? "view" : "table";
        if (s.if_flag) o += " if-exists";
        o += ' ';
        name(o, s.name);
        o += ')';
        break;
      case StmtKind::Optimize:
        o += "(optimize ";
        name(o, s.name);
        if (s.value) {
          o += ' ';
          expr(*s.value);
        }
        o += ')';
        break;
      case StmtKind::Set:
        o += "(set ";
        name(o, s.name);
        o += ' ';
        expr(*s.value);
        o += ')';
        break;
    }
  }
};

}  // namespace

std::string dump(const Statement &s) {
  D d;
  d.stmt(s);
  return std::move(d.o);
}

std::string dump(const Expr &e) {
  D d;
  d.expr(e);
  return std::move(d.o);
}

}  // namespace nut::sql
