// jit.cpp — query-specific scan kernels.
//
// A query whose WHERE / aggregate arguments are not one of the precompiled shapes
// (agg_ops.hpp: Fixed<>) arrives as expression programs (nut_prog: RPN node arrays,
// include/nutexec.h).  They are type-checked here and turned into straight-line device
// code — a kProg shape struct whose where()/value()/valid() the streaming kernel
// (agg_kernel.hpp) inlines into its per-row loop — and compiled with hipRTC for gfx950
// against the same kernel template the precompiled shapes use.  So an arbitrary
// expression costs the same per row as a hand-instantiated shape: no interpreter, no
// per-row dispatch.
//   * constants live in the kernel arguments (AggArgs::kc), not in the source, so
//     queries that differ only in constants share one code object;
//   * code objects are cached per translation unit (process-wide) and modules per
//     device; a first compile takes about a second;
//   * the kernel headers are embedded at build time (_gen/jit_headers.inc, written by
//     nutdb_amd/build.py), so the library needs no source tree at run time.
#include "jit.hpp"

#include <hip/hiprtc.h>
#include <string.h>

#include <map>
#include <mutex>

namespace nut {
namespace {

#include "_gen/jit_headers.inc"  // kJitHeaders[][2] = {name, text}

// ------------------------------------------------------------------ type check + codegen
struct PVal {
  int t;          // nut_prog_value_type
  std::string s;  // C++ expression text
};

struct Gen {
  const int32_t *col_types;
  int ncols;
  std::vector<uint64_t> *consts;
  std::string err;

  bool fail(const std::string &m) {
    if (err.empty()) err = m;
    return false;
  }
  std::string konst(uint64_t bits) {
    size_t i = 0;
    while (i < consts->size() && (*consts)[i] != bits) ++i;
    if (i == consts->size()) consts->push_back(bits);
    return "p.kc[" + std::to_string(i) + "]";
  }
  static std::string as_i(const PVal &v) { return v.t == NUT_PT_BOOL ? "((int64_t)" + v.s + ")" : v.s; }
  static std::string as_f(const PVal &v) { return v.t == NUT_PT_F64 ? v.s : "((double)" + as_i(v) + ")"; }
  bool as_b(const PVal &v, std::string &out, const char *what) {
    if (v.t == NUT_PT_F64) return fail(std::string(what) + " needs a boolean or integer operand, got float64");
    out = v.t == NUT_PT_BOOL ? v.s : "(" + v.s + " != 0)";
    return true;
  }

  bool run(const nut_prog *p, PVal &res) {
    if (!p || p->n <= 0) return fail("empty expression program");
    if (p->n > NUT_MAX_PROG_NODES) return fail("expression program longer than 256 nodes");
    if (!p->node) return fail("expression program has no nodes");
    std::vector<PVal> st;
    auto pop = [&](int k, PVal *o) {
      if ((int)st.size() < k) return false;
      for (int i = k - 1; i >= 0; --i) {
        o[i] = std::move(st.back());
        st.pop_back();
      }
      return true;
    };
    for (int i = 0; i < p->n; ++i) {
      const nut_prog_node &nd = p->node[i];
      PVal a[3];
      const int op = nd.op;
      const int arity = op <= NUT_P_F64 ? 0 : (op == NUT_P_NOT || op == NUT_P_BITNOT || op == NUT_P_ABS ||
                                                op == NUT_P_TO_F64 || op == NUT_P_LOOKUP || op == NUT_P_DATEPART || op == NUT_P_MAP) ? 1
                                                                                         : op == NUT_P_IF ? 3 : 2;
      if (op < 0 || op > NUT_P_MAP) return fail("unknown program op " + std::to_string(op));
      if (!pop(arity, a)) return fail("program stack underflow at node " + std::to_string(i));
      PVal r;
      const bool f = arity == 2 && (a[0].t == NUT_PT_F64 || a[1].t == NUT_PT_F64);
      std::string b0, b1, b2;
      switch (op) {
        case NUT_P_COL:
          if (nd.arg < 0 || nd.arg >= ncols) return fail("program column index out of range");
          if (col_types[nd.arg] == NUT_T_F64) r = {NUT_PT_F64, "as_f64(v[" + std::to_string(nd.arg) + "][r])"};
          else r = {NUT_PT_I64, "((int64_t)v[" + std::to_string(nd.arg) + "][r])"};
          break;
        case NUT_P_I64: r = {NUT_PT_I64, "((int64_t)" + konst((uint64_t)nd.v) + ")"}; break;
        case NUT_P_F64: r = {NUT_PT_F64, "as_f64(" + konst((uint64_t)nd.v) + ")"}; break;
        case NUT_P_ADD:
        case NUT_P_SUB:
        case NUT_P_MUL: {
          const char *o = op == NUT_P_ADD ? " + " : op == NUT_P_SUB ? " - " : " * ";
          if (f) r = {NUT_PT_F64, "(" + as_f(a[0]) + o + as_f(a[1]) + ")"};
          else r = {NUT_PT_I64, "((int64_t)((uint64_t)" + as_i(a[0]) + o + "(uint64_t)" + as_i(a[1]) + "))"};
          break;
        }
        case NUT_P_DIV: r = {NUT_PT_F64, "(" + as_f(a[0]) + " / " + as_f(a[1]) + ")"}; break;
        case NUT_P_MOD:
          if (f) r = {NUT_PT_F64, "fmod(" + as_f(a[0]) + ", " + as_f(a[1]) + ")"};
          else r = {NUT_PT_I64, "jmod(" + as_i(a[0]) + ", " + as_i(a[1]) + ", err)"};
          break;
        case NUT_P_INTDIV:
          if (f) return fail("integer division needs integer operands");
          r = {NUT_PT_I64, "jdiv(" + as_i(a[0]) + ", " + as_i(a[1]) + ", err)"};
          break;
        case NUT_P_LT:
        case NUT_P_LE:
        case NUT_P_GT:
        case NUT_P_GE:
        case NUT_P_EQ:
        case NUT_P_NE: {
          static const char *cmp[] = {" < ", " <= ", " > ", " >= ", " == ", " != "};
          const char *o = cmp[op - NUT_P_LT];
          r = {NUT_PT_BOOL, f ? "(" + as_f(a[0]) + o + as_f(a[1]) + ")" : "(" + as_i(a[0]) + o + as_i(a[1]) + ")"};
          break;
        }
        case NUT_P_AND:
        case NUT_P_OR:
        case NUT_P_XOR: {
          const char *o = op == NUT_P_AND ? " & " : op == NUT_P_OR ? " | " : " != ";
          if (!as_b(a[0], b0, "AND/OR/XOR") || !as_b(a[1], b1, "AND/OR/XOR")) return false;
          r = {NUT_PT_BOOL, "((bool)(" + b0 + o + b1 + "))"};
          break;
        }
        case NUT_P_NOT:
          if (!as_b(a[0], b0, "NOT")) return false;
          r = {NUT_PT_BOOL, "(!" + b0 + ")"};
          break;
        case NUT_P_BITAND:
        case NUT_P_BITOR:
        case NUT_P_BITXOR:
        case NUT_P_SHL:
        case NUT_P_SHR: {
          if (f) return fail("bitwise operators need integer operands");
          if (op == NUT_P_SHL || op == NUT_P_SHR) {
            r = {NUT_PT_I64, std::string(op == NUT_P_SHL ? "jshl(" : "jshr(") + as_i(a[0]) + ", " + as_i(a[1]) + ")"};
          } else {
            const char *o = op == NUT_P_BITAND ? " & " : op == NUT_P_BITOR ? " | " : " ^ ";
            r = {NUT_PT_I64, "(" + as_i(a[0]) + o + as_i(a[1]) + ")"};
          }
          break;
        }
        case NUT_P_BITNOT:
          if (a[0].t == NUT_PT_F64) return fail("bitwise operators need integer operands");
          r = {NUT_PT_I64, "(~" + as_i(a[0]) + ")"};
          break;
        case NUT_P_IF: {
          if (!as_b(a[0], b0, "IF condition")) return false;
          const PVal &x = a[1], &y = a[2];
          if (x.t == NUT_PT_BOOL && y.t == NUT_PT_BOOL) r = {NUT_PT_BOOL, "(" + b0 + " ? " + x.s + " : " + y.s + ")"};
          else if (x.t == NUT_PT_F64 || y.t == NUT_PT_F64)
            r = {NUT_PT_F64, "(" + b0 + " ? " + as_f(x) + " : " + as_f(y) + ")"};
          else r = {NUT_PT_I64, "(" + b0 + " ? " + as_i(x) + " : " + as_i(y) + ")"};
          break;
        }
        case NUT_P_ABS:
          r = a[0].t == NUT_PT_F64 ? PVal{NUT_PT_F64, "fabs(" + a[0].s + ")"}
                                   : PVal{NUT_PT_I64, "jabs(" + as_i(a[0]) + ")"};
          break;
        case NUT_P_TO_F64: r = {NUT_PT_F64, as_f(a[0])}; break;
        case NUT_P_LOOKUP:
          if (a[0].t == NUT_PT_F64) return fail("LOOKUP needs an integer operand");
          if (nd.arg < 0) return fail("LOOKUP table length is negative");
          if (nd.arg > 0 && nd.v == 0) return fail("LOOKUP table has no address");
          r = {NUT_PT_BOOL, "jlookup(" + as_i(a[0]) + ", " + konst((uint64_t)nd.v) + ", " +
                                konst((uint64_t)(int64_t)nd.arg) + ")"};
          break;
        case NUT_P_MAP:
          if (a[0].t == NUT_PT_F64) return fail("MAP needs an integer operand");
          if (nd.arg < 0) return fail("MAP table length is negative");
          if (nd.arg > 0 && nd.v == 0) return fail("MAP table has no address");
          r = {NUT_PT_I64, "jmap(" + as_i(a[0]) + ", " + konst((uint64_t)nd.v) + ", " +
                               konst((uint64_t)(int64_t)nd.arg) + ")"};
          break;
        case NUT_P_DATEPART:
          if (a[0].t == NUT_PT_F64) return fail("DATEPART needs an integer operand (days)");
          if (nd.arg < NUT_DP_YEAR || nd.arg > NUT_DP_YYYYMMDD) return fail("DATEPART: unknown part " + std::to_string(nd.arg));
          r = {NUT_PT_I64, "jdatepart(" + as_i(a[0]) + ", " + std::to_string(nd.arg) + ")"};
          break;
      }
      if (r.s.size() > (1u << 20)) return fail("expression program too large");
      st.push_back(std::move(r));
    }
    if (st.size() != 1) return fail("expression program leaves " + std::to_string(st.size()) + " values (want 1)");
    res = std::move(st.back());
    return true;
  }
};

const char *kPrelude = R"(// generated by nutexec jit.cpp
typedef unsigned long uint64_t;
typedef long int64_t;
typedef unsigned int uint32_t;
typedef int int32_t;
typedef unsigned short uint16_t;
typedef unsigned char uint8_t;
#include "agg_kernel.hpp"
#include "select_kernel.hpp"
namespace nut {
// integer helpers of the expression semantics (include/nutexec.h, nut_prog_op)
__device__ __forceinline__ int64_t jmod(int64_t a, int64_t b, bool &err) {
  if (b == 0) { err = true; return 0; }
  return b == -1 ? 0 : a % b;
}
__device__ __forceinline__ int64_t jdiv(int64_t a, int64_t b, bool &err) {
  if (b == 0) { err = true; return 0; }
  return b == -1 ? (int64_t)(0 - (uint64_t)a) : a / b;
}
__device__ __forceinline__ int64_t jshl(int64_t a, int64_t b) {
  return (b >= 0 && b < 64) ? (int64_t)((uint64_t)a << b) : 0;
}
__device__ __forceinline__ int64_t jshr(int64_t a, int64_t b) {
  return (b >= 0 && b < 64) ? (a >> b) : (a < 0 ? -1 : 0);
}
__device__ __forceinline__ int64_t jabs(int64_t a) { return a < 0 ? (int64_t)(0 - (uint64_t)a) : a; }
// byte-table membership; an empty table (n == 0) is never read
__device__ __forceinline__ bool jlookup(int64_t x, uint64_t t, uint64_t n) {
  if ((uint64_t)x >= n) return false;
  return ((const uint8_t *)t)[x] != 0;
}
// int64-table map (code -> code); outside the table: -1, which no dictionary string has
__device__ __forceinline__ int64_t jmap(int64_t x, uint64_t t, uint64_t n) {
  if ((uint64_t)x >= n) return -1;
  return ((const int64_t *)t)[x];
}
// civil-from-days (proleptic Gregorian); P = nut_date_part.  d is clamped to +-2^40 days
// first, so no intermediate overflows.
__device__ __forceinline__ int64_t jdatepart(int64_t d, const int P) {
  d = d < -(1ll << 40) ? -(1ll << 40) : d > (1ll << 40) ? (1ll << 40) : d;
  const int64_t z = d + 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);  // from March 1
  const int64_t mp = (5 * doy + 2) / 153;
  const int64_t m = mp < 10 ? mp + 3 : mp - 9;
  const int64_t y = yoe + era * 400 + (m <= 2 ? 1 : 0);
  if (P == 0) return y;
  if (P == 1) return m;
  if (P == 2) return doy - (153 * mp + 2) / 5 + 1;
  if (P == 6) return y * 100 + m;
  if (P == 7) return y * 10000 + m * 100 + (doy - (153 * mp + 2) / 5 + 1);
  if (P == 3) return (m - 1) / 3 + 1;
  if (P == 4) {  // 1970-01-01 was a Thursday (4)
    int64_t w = d % 7;
    w = w < 0 ? w + 7 : w;
    return (w + 3) % 7 + 1;
  }
  // day of year: January / February are days 306.. of the March-based year
  return doy >= 306 ? doy - 305 : doy + 60 + (((y % 4 == 0 && y % 100 != 0) || y % 400 == 0) ? 1 : 0);
}
)";

std::string bits_of(const PVal &v) {
  return v.t == NUT_PT_F64 ? "as_u64(" + v.s + ")" : "(uint64_t)" + Gen::as_i(v);
}

// ------------------------------------------------------------------ compile cache
std::mutex g_mu;
std::map<std::string, std::vector<char>> g_code;                      // unit -> code object
std::map<std::pair<int, std::string>, std::pair<hipModule_t, hipFunction_t>> g_fn;  // (device, unit)

nut_status compile_unit(const std::string &unit, const std::vector<char> *&code) {
  auto it = g_code.find(unit);
  if (it != g_code.end()) {
    code = &it->second;
    return NUT_OK;
  }
  const int nh = (int)(sizeof(kJitHeaders) / sizeof(kJitHeaders[0]));
  std::vector<const char *> hdr(nh), names(nh);
  for (int i = 0; i < nh; ++i) names[i] = kJitHeaders[i][0], hdr[i] = kJitHeaders[i][1];
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, unit.c_str(), "nut_jit_scan.hip", nh, hdr.data(), names.data()) != HIPRTC_SUCCESS)
    return fail(NUT_ERR_HIP, "hiprtcCreateProgram failed");
  // the expression marker after "// kernel " names the instantiation to look up
  const size_t k = unit.rfind("// kernel ");
  const std::string expr = unit.substr(k + 10, unit.find('\n', k) - k - 10);
  hiprtcAddNameExpression(prog, expr.c_str());
  const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-munsafe-fp-atomics"};
  hiprtcResult rc = hiprtcCompileProgram(prog, (int)(sizeof(opts) / sizeof(opts[0])), opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    return fail(NUT_ERR_HIP, "hipRTC compile of the expression kernel failed: " + log.substr(0, 4000));
  }
  const char *lowered = nullptr;
  hiprtcGetLoweredName(prog, expr.c_str(), &lowered);
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  std::vector<char> obj(cs + 512);
  hiprtcGetCode(prog, obj.data());
  // keep the lowered (mangled) name after the code object, NUL-separated
  const std::string ln = lowered ? lowered : "";
  obj.resize(cs);
  obj.push_back('\0');
  obj.insert(obj.end(), ln.begin(), ln.end());
  obj.push_back('\0');
  hiprtcDestroyProgram(&prog);
  if (ln.empty()) return fail(NUT_ERR_HIP, "hipRTC: no lowered name for " + expr);
  code = &(g_code[unit] = std::move(obj));
  return NUT_OK;
}

}  // namespace

nut_status prog_check(const nut_prog *p, const int32_t *col_types, int ncols, int32_t *type) {
  std::vector<uint64_t> consts;
  Gen g{col_types, ncols, &consts, {}};
  PVal r;
  if (!g.run(p, r)) return fail(NUT_ERR_INVALID_ARG, "nut_prog: " + g.err);
  *type = r.t;
  return NUT_OK;
}

nut_status jit_shape(const nut_agg_spec *s, const int32_t *kinds, JitShape &out) {
  out.consts.clear();
  Gen g{s->prog_col_type, s->nprog_cols, &out.consts, {}};
  std::string where = "true", value, valid;
  PVal r;
  if (s->where.n) {
    if (!g.run(&s->where, r)) return fail(NUT_ERR_INVALID_ARG, "nut_groupby WHERE program: " + g.err);
    if (!g.as_b(r, where, "WHERE")) return fail(NUT_ERR_INVALID_ARG, "nut_groupby WHERE program: " + g.err);
  }
  for (int a = 0; a < s->naggs; ++a) {
    out.types[a] = NUT_PT_I64;
    const std::string ca = "      case " + std::to_string(a) + ": return ";
    if (s->agg_op[a] != NUT_AGG_COUNT) {
      if (!g.run(&s->agg_val[a], r))
        return fail(NUT_ERR_INVALID_ARG, "nut_groupby aggregate " + std::to_string(a) + " program: " + g.err);
      out.types[a] = r.t;
      value += ca + bits_of(r) + ";\n";
    }
    if (s->agg_mask[a].n) {
      std::string b;
      if (!g.run(&s->agg_mask[a], r) || !g.as_b(r, b, "aggregate mask"))
        return fail(NUT_ERR_INVALID_ARG, "nut_groupby aggregate " + std::to_string(a) + " mask: " + g.err);
      valid += ca + b + ";\n";
    }
  }
  // computed keys (nut_agg_spec.key_prog): int64 / bool programs
  std::string keys;
  int kmask = 0;
  for (int j = 0; j < s->nkeys && j < NUT_MAX_KEYS; ++j) {
    if (!s->key_prog[j].n) continue;
    if (!g.run(&s->key_prog[j], r)) return fail(NUT_ERR_INVALID_ARG, "nut_groupby key " + std::to_string(j) + " program: " + g.err);
    if (r.t == NUT_PT_F64) return fail(NUT_ERR_INVALID_ARG, "nut_groupby key " + std::to_string(j) + " program: float64 keys are not grouped");
    keys += "      case " + std::to_string(j) + ": return " + bits_of(r) + ";\n";
    kmask |= 1 << j;
  }
  uint32_t kp = 0;
  for (int a = 0; a < s->naggs; ++a) kp |= (uint32_t)(kinds[a] & 15) << (4 * a);
  const int ma = s->naggs > 0 ? s->naggs : 1;
  std::string src;
  src += "struct QShape {\n";
  src += "  static constexpr bool kProg = true;\n";
  src += "  static constexpr int MP = 0, MV = " + std::to_string(s->nprog_cols) + ", MA = " + std::to_string(ma) + ";\n";
  src += "  static constexpr uint32_t kKinds = " + std::to_string(kp) + "u;\n";
  src += "  static constexpr int kKeyProg = " + std::to_string(kmask) + ";\n";
  src += "  __device__ static constexpr int np(const AggArgs &) { return 0; }\n";
  src += "  __device__ static constexpr int nv(const AggArgs &) { return MV; }\n";
  src += "  __device__ static constexpr int na(const AggArgs &) { return " + std::to_string(s->naggs) + "; }\n";
  src += "  __device__ static constexpr int kind(const AggArgs &, int a) { return (int)((kKinds >> (4 * a)) & 15u); }\n";
  src += "  __device__ static constexpr int expr(const AggArgs &, int) { return 0; }\n";
  src += "  __device__ static constexpr int arg(const AggArgs &, int, int) { return 0; }\n";
  src += "  __device__ static constexpr int ptype(const AggArgs &, int) { return 0; }\n";
  src += "  __device__ static constexpr int pop(const AggArgs &, int) { return 0; }\n";
  src += "  template <class V>\n  __device__ __forceinline__ static bool where(const AggArgs &p, const V &v, int r, bool &err) {\n";
  src += "    return " + where + ";\n  }\n";
  src += "  template <class V>\n  __device__ __forceinline__ static uint64_t value(const AggArgs &p, int a, const V &v, int r, bool &err) {\n";
  src += "    switch (a) {\n" + value + "      default: return 0;\n    }\n  }\n";
  src += "  template <class V>\n  __device__ __forceinline__ static bool valid(const AggArgs &p, int a, const V &v, int r, bool &err) {\n";
  src += "    switch (a) {\n" + valid + "      default: return true;\n    }\n  }\n";
  src += "  template <class V>\n  __device__ __forceinline__ static uint64_t key(const AggArgs &p, int j, const V &v, int r, bool &err) {\n";
  src += "    switch (j) {\n" + keys + "      default: return 0;\n    }\n  }\n";
  src += "};\n";
  out.src = std::move(src);
  return NUT_OK;
}

std::string jit_unit(const std::string &shape_src, int nk, bool priv, int bd, size_t args_size) {
  std::string u = kPrelude;
  u += "static_assert(sizeof(AggArgs) == " + std::to_string(args_size) + ", \"AggArgs layout\");\n";
  u += shape_src;
  const std::string inst = "agg_kernel<" + std::to_string(nk) + ", " + (priv ? "true" : "false") + ", " +
                           std::to_string(bd) + ", nut::QShape, 0>";
  u += "template __global__ void " + inst + "(AggArgs);\n}  // namespace nut\n";
  u += "// kernel &nut::" + inst + "\n";
  return u;
}

std::string jit_select_unit(const std::string &shape_src, size_t args_size) {
  std::string u = kPrelude;
  u += "static_assert(sizeof(SelArgs) == " + std::to_string(args_size) + ", \"SelArgs layout\");\n";
  u += shape_src;
  u += "template __global__ void select_kernel<nut::QShape>(SelArgs);\n}  // namespace nut\n";
  u += "// kernel &nut::select_kernel<nut::QShape>\n";
  return u;
}

std::string jit_eval_unit(const std::string &shape_src, size_t args_size) {
  std::string u = kPrelude;
  u += "static_assert(sizeof(EvalArgs) == " + std::to_string(args_size) + ", \"EvalArgs layout\");\n";
  u += shape_src;
  u += "template __global__ void eval_kernel<nut::QShape>(EvalArgs);\n}  // namespace nut\n";
  u += "// kernel &nut::eval_kernel<nut::QShape>\n";
  return u;
}

nut_status jit_kernel(const std::string &unit, bool load, hipFunction_t *fn) {
  std::lock_guard<std::mutex> lk(g_mu);
  int dev = 0;
  if (load) NUT_HIP(hipGetDevice(&dev));
  if (load) {
    auto it = g_fn.find({dev, unit});
    if (it != g_fn.end()) {
      *fn = it->second.second;
      return NUT_OK;
    }
  }
  const std::vector<char> *code = nullptr;
  nut_status st = compile_unit(unit, code);
  if (st || !load) return st;
  // code object, NUL, lowered name, NUL
  const char *name = code->data() + code->size() - 2;
  while (name > code->data() && name[-1] != '\0') --name;
  hipModule_t mod;
  NUT_HIP(hipModuleLoadData(&mod, code->data()));
  hipFunction_t f;
  hipError_t e = hipModuleGetFunction(&f, mod, name);
  if (e != hipSuccess) {
    (void)hipModuleUnload(mod);
    return hip_fail(e, "hipModuleGetFunction (expression kernel)");
  }
  g_fn[{dev, unit}] = {mod, f};
  *fn = f;
  return NUT_OK;
}

}  // namespace nut

extern "C" nut_status nut_prog_type(const nut_prog *prog, const int32_t *col_types, int ncols, int32_t *type) {
  if (!prog || !type || (ncols && !col_types) || ncols < 0 || ncols > NUT_MAX_PROG_COLS)
    return nut::fail(NUT_ERR_INVALID_ARG, "nut_prog_type: bad argument");
  return nut::prog_check(prog, col_types, ncols, type);
}
