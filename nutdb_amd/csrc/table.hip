// table.hip — typed device tables from CREATE TABLE (table.hpp).
//
// nut_table_create maps the reference's column types (ast/item.rs:14-68) to HBM columns;
// nut_table_append moves host values to HBM at their declared width and widens them
// there (one streaming kernel: sign/zero extension, Float32 -> f64, Boolean -> 0/1), so
// the PCIe transfer carries the narrow bytes.  String-like columns are dictionary-encoded
// on the host (the dictionary is what binds string constants at plan time) and their
// int64 codes feed the same hash / compare paths as any other int64 column.
#include <string.h>

#include <algorithm>

#include "sql_ast.hpp"
#include "table.hpp"

using namespace nut;

namespace {

// one launch widens n host-width values into int64 / f64 words; bit 0 of *bad: a UInt64
// value >= 2^63 (not representable in the int64 execution type)
__global__ void widen_kernel(const uint8_t *__restrict__ src, uint64_t *__restrict__ dst, uint64_t n, int width,
                             int kind, uint32_t *bad) {
  bool b = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t w;
    if (kind == NUT_COL_FLOAT) {
      if (width == 4) {
        float f;
        memcpy(&f, src + i * 4, 4);
        w = as_u64((double)f);
      } else {
        memcpy(&w, src + i * 8, 8);
      }
    } else if (kind == NUT_COL_BOOL) {
      w = src[i] != 0;
    } else {
      const bool sgn = kind == NUT_COL_INT;
      switch (width) {
        case 1: w = sgn ? (uint64_t)(int64_t)(int8_t)src[i] : (uint64_t)src[i]; break;
        case 2: {
          uint16_t v;
          memcpy(&v, src + i * 2, 2);
          w = sgn ? (uint64_t)(int64_t)(int16_t)v : (uint64_t)v;
          break;
        }
        case 4: {
          uint32_t v;
          memcpy(&v, src + i * 4, 4);
          w = sgn ? (uint64_t)(int64_t)(int32_t)v : (uint64_t)v;
          break;
        }
        default:
          memcpy(&w, src + i * 8, 8);
          b = b || (!sgn && (w >> 63));
      }
    }
    dst[i] = w;
  }
  if (b) atomicOr(bad, 1u);
}

bool map_type(const sql::DataType &t, TCol &c, std::string &err) {
  using sql::Compound;
  using sql::Scalar;
  if (!t.scalar) {
    switch (t.c) {
      case Compound::Nullable:
      case Compound::Dictionary:  // a dictionary of strings is how strings execute anyway
        return map_type(t.kids[0], c, err);
      case Compound::Enum:
        c.kind = NUT_COL_ENUM;
        c.own.fixed = true;
        for (const auto &b : t.binds) {
          if (b.id > (uint64_t)INT64_MAX) return err = "Enum id out of range", false;
          c.own.codes[b.literal] = (int64_t)b.id;
        }
        c.dict = &c.own;
        return true;
      default:
        err = "Array / Tuple / Map columns are not executed";
        return false;
    }
  }
  c.exec_type = NUT_T_I64;
  switch (t.s) {
    case Scalar::Int8: c.kind = NUT_COL_INT, c.width = 1; return true;
    case Scalar::Int16: c.kind = NUT_COL_INT, c.width = 2; return true;
    case Scalar::Int32:
    case Scalar::Serial32: c.kind = NUT_COL_INT, c.width = 4; return true;
    case Scalar::Int64:
    case Scalar::Serial64: c.kind = NUT_COL_INT, c.width = 8; return true;
    case Scalar::UInt8: c.kind = NUT_COL_UINT, c.width = 1; return true;
    case Scalar::UInt16: c.kind = NUT_COL_UINT, c.width = 2; return true;
    case Scalar::UInt32:
    case Scalar::USerial32: c.kind = NUT_COL_UINT, c.width = 4; return true;
    case Scalar::UInt64:
    case Scalar::USerial64: c.kind = NUT_COL_UINT, c.width = 8; return true;
    case Scalar::Float32: c.kind = NUT_COL_FLOAT, c.width = 4, c.exec_type = NUT_T_F64; return true;
    case Scalar::Float64: c.kind = NUT_COL_FLOAT, c.width = 8, c.exec_type = NUT_T_F64; return true;
    case Scalar::Boolean: c.kind = NUT_COL_BOOL, c.width = 1; return true;
    case Scalar::Date: c.kind = NUT_COL_DATE, c.width = 8; return true;
    case Scalar::Datetime: c.kind = NUT_COL_DATETIME, c.width = 8; return true;
    case Scalar::Chars:
    case Scalar::String: c.kind = NUT_COL_STRING, c.width = 0; return true;
    default:
      err = "128-bit integers, Decimal and Uuid columns are not executed (int64 / f64 execution types)";
      return false;
  }
}

nut_status grow(nut_ctx *c, TCol &col, uint64_t need) {
  if (need <= col.cap) return NUT_OK;
  uint64_t cap = col.cap ? col.cap : 1024;
  while (cap < need) cap *= 2;
  void *p = nullptr;
  NUT_HIP(hipMalloc(&p, cap * 8));
  if (col.n) {
    hipError_t e = hipMemcpyAsync(p, col.dev, col.n * 8, hipMemcpyDeviceToDevice, c->stream);
    if (e != hipSuccess) {
      (void)hipFree(p);
      return hip_fail(e, "nut_table_append: grow");
    }
    NUT_HIP(hipStreamSynchronize(c->stream));
  }
  if (col.dev) (void)hipFree(col.dev);
  col.dev = p;
  col.cap = cap;
  return NUT_OK;
}

}  // namespace

extern "C" {

nut_status nut_table_create(const char *sql, size_t len, nut_table **out) {
  if (!out || (!sql && len)) return fail(NUT_ERR_INVALID_ARG, "nut_table_create: NULL argument");
  *out = nullptr;
  const std::string text(sql ? sql : "", len);
  sql::Statement st;
  sql::ParseError pe;
  if (!sql::parse(sql::sv(text), st, pe)) return fail(NUT_ERR_PARSE, pe.str());
  if (st.k != sql::StmtKind::Create || st.is_view || !st.table)
    return fail(NUT_ERR_INVALID_ARG, "nut_table_create: expected CREATE TABLE");
  nut_table *t = new nut_table;
  t->name = std::string(st.table->name);
  for (const auto &cd : st.table->columns) {
    TCol c;
    c.name = std::string(cd.name);
    std::string err;
    if (!map_type(cd.t, c, err)) {
      delete t;
      return fail(NUT_ERR_UNSUPPORTED, "column '" + c.name + "': " + err);
    }
    for (const auto &o : t->cols)
      if (o.name == c.name) {
        delete t;
        return fail(NUT_ERR_INVALID_ARG, "duplicate column '" + c.name + "'");
      }
    t->cols.push_back(std::move(c));
  }
  // string columns share the table dictionary (codes compare across columns); Enum
  // columns point at their own (the vector is final, so the pointers stay valid)
  for (auto &c : t->cols) c.dict = c.kind == NUT_COL_STRING ? &t->strings : c.kind == NUT_COL_ENUM ? &c.own : nullptr;
  if (t->cols.empty()) {
    delete t;
    return fail(NUT_ERR_INVALID_ARG, "nut_table_create: no columns");
  }
  *out = t;
  return NUT_OK;
}

nut_status nut_table_shape(const nut_table *t, int *ncols, uint64_t *nrows) {
  if (!t) return fail(NUT_ERR_INVALID_ARG, "nut_table_shape: NULL table");
  if (ncols) *ncols = (int)t->cols.size();
  if (nrows) *nrows = t->rows();
  return NUT_OK;
}

nut_status nut_table_column_info(const nut_table *t, int j, const char **name, int *kind, int *width,
                                 int *exec_type) {
  if (!t || j < 0 || j >= (int)t->cols.size()) return fail(NUT_ERR_INVALID_ARG, "nut_table_column_info: bad column");
  const TCol &c = t->cols[j];
  if (name) *name = c.name.c_str();
  if (kind) *kind = c.kind;
  if (width) *width = c.width;
  if (exec_type) *exec_type = c.exec_type;
  return NUT_OK;
}

nut_status nut_table_append(nut_ctx *c, nut_table *t, int j, const void *data, const int64_t *offsets, uint64_t n) {
  if (!c || !t || j < 0 || j >= (int)t->cols.size()) return fail(NUT_ERR_INVALID_ARG, "nut_table_append: bad argument");
  if (n == 0) return NUT_OK;
  if (!data && !(offsets && offsets[n] == offsets[0])) return fail(NUT_ERR_INVALID_ARG, "nut_table_append: NULL data");
  if (t->device >= 0 && t->device != c->device)
    return fail(NUT_ERR_INVALID_ARG, "nut_table_append: the table lives on another device");
  DeviceGuard dg(c->device);
  TCol &col = t->cols[j];
  nut_status st = grow(c, col, col.n + n);
  if (st) return st;
  t->device = c->device;
  uint64_t *dst = (uint64_t *)col.dev + col.n;
  if (col.kind == NUT_COL_STRING || col.kind == NUT_COL_ENUM) {
    if (!offsets) return fail(NUT_ERR_INVALID_ARG, "nut_table_append: string columns take offsets");
    std::vector<int64_t> codes(n);
    Dict &d = *col.dict;
    for (uint64_t i = 0; i < n; ++i) {
      if (offsets[i + 1] < offsets[i]) return fail(NUT_ERR_INVALID_ARG, "nut_table_append: offsets decrease");
      std::string s((const char *)data + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
      int64_t code = d.find(s);
      if (code < 0) {
        if (d.fixed) return fail(NUT_ERR_INVALID_ARG, "column '" + col.name + "': '" + s + "' is not a value of its Enum");
        code = d.intern(std::move(s));
      }
      codes[i] = code;
    }
    NUT_HIP(hipMemcpyAsync(dst, codes.data(), n * 8, hipMemcpyHostToDevice, c->stream));
    NUT_HIP(hipStreamSynchronize(c->stream));
  } else if (col.width == 8 && col.kind != NUT_COL_UINT) {
    NUT_HIP(hipMemcpyAsync(dst, data, n * 8, hipMemcpyHostToDevice, c->stream));
    NUT_HIP(hipStreamSynchronize(c->stream));
  } else {
    // narrow bytes over PCIe, widened in HBM (staged through ctx scratch in chunks)
    const uint64_t chunk = (64ull << 20) / (uint64_t)col.width;
    const size_t sbytes = (size_t)std::min(n, chunk) * (size_t)col.width;
    nut_status s2 = c->misc.reserve(sbytes + 256);
    if (s2) return s2;
    uint8_t *stage = (uint8_t *)c->misc.ptr;
    uint32_t *bad = (uint32_t *)(stage + ((sbytes + 15) & ~size_t(15)));
    NUT_HIP(hipMemsetAsync(bad, 0, 4, c->stream));
    for (uint64_t i0 = 0; i0 < n; i0 += chunk) {
      const uint64_t m = std::min(chunk, n - i0);
      NUT_HIP(hipMemcpyAsync(stage, (const uint8_t *)data + i0 * col.width, m * col.width, hipMemcpyHostToDevice,
                             c->stream));
      const uint64_t blocks = std::min<uint64_t>((m + 255) / 256, (uint64_t)c->num_cus * 8);
      hipLaunchKernelGGL(widen_kernel, dim3((unsigned)blocks), dim3(256), 0, c->stream, stage, dst + i0, m,
                         col.width, col.kind, bad);
      NUT_HIP(hipGetLastError());
    }
    uint32_t flag = 0;
    NUT_HIP(hipMemcpyAsync(&flag, bad, 4, hipMemcpyDeviceToHost, c->stream));
    NUT_HIP(hipStreamSynchronize(c->stream));
    if (flag) return fail(NUT_ERR_UNSUPPORTED, "column '" + col.name + "': UInt64 values >= 2^63 are not executed");
  }
  col.n += n;
  return NUT_OK;
}

void nut_table_free(nut_table *t) {
  if (!t) return;
  for (auto &c : t->cols)
    if (c.dev) (void)hipFree(c.dev);
  delete t;
}

}  // extern "C"
