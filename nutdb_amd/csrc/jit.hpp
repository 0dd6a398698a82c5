// jit.hpp — query-specific scan kernels: expression programs
// (nut_prog, RPN) -> a generated kProg shape -> hipRTC -> the agg_kernel template.
#pragma once

#include <string>
#include <vector>

#include "common.hpp"

namespace nut {

struct JitShape {
  std::string src;              // shape source (constants are NOT in it)
  std::vector<uint64_t> consts; // kernel-argument constants, AggArgs::kc order
  int32_t types[NUT_MAX_AGGS];  // nut_prog_value_type of each aggregate argument
};

// type-check a program: *type = nut_prog_value_type, or a failed status with the reason
nut_status prog_check(const nut_prog *p, const int32_t *col_types, int ncols, int32_t *type);
// type-check every program of an expression-mode spec and generate its shape
nut_status jit_shape(const nut_agg_spec *s, const int32_t *kinds, JitShape &out);
// the full translation unit of one kernel variant
// (args_size = sizeof(AggArgs) on the host: the unit asserts the same layout)
std::string jit_unit(const std::string &shape_src, int nk, bool priv, int bd, size_t args_size);
// the translation unit of the expression-mode scan (select_kernel.hpp) for a shape
std::string jit_select_unit(const std::string &shape_src, size_t args_size);
std::string jit_eval_unit(const std::string &shape_src, size_t args_size);
// compile (cached per unit) and, when load is set, load on the current device
nut_status jit_kernel(const std::string &unit, bool load, hipFunction_t *fn);

}  // namespace nut
