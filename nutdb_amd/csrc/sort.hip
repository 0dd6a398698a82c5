// sort.hip — SELECT k FROM t ORDER BY k  (BASELINE config 5)
#include "common.hpp"

using namespace nut;

extern "C" nut_status nut_sort_i64(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n) {
  if (!c || (n && (!in || !out))) return fail(NUT_ERR_INVALID_ARG, "nut_sort_i64: NULL argument");
  return fail(NUT_ERR_UNSUPPORTED, "nut_sort_i64: not implemented yet");
}
