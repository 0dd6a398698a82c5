// sort.hpp — internal entry points shared between translation units: the two sort
// implementations behind nut_sort_i64 / nut_sort_i64_desc, and join helpers.
// Both take validated arguments (n > 0, in != out, device set) and `flip`, the XOR that maps
// int64 order to unsigned order (ascending) or to its reverse (descending).
#pragma once

#include <vector>
#include "common.hpp"

namespace nut {
// bounds (optional): {lo, hi} such that every key k satisfies lo <= k ^ flip <= hi (a
// sample-sort rank's splitter range); the capped layout then spreads exactly that range
nut_status msd_sort_i64(nut_ctx *c, const int64_t *in, int64_t *out, uint64_t n, uint64_t flip,
                        const uint64_t *bounds = nullptr);  // msd_sort.hip
// unstable range partition by <= 63 ascending splitters (the sample sort's send layout)
nut_status partition_i64_ranges(nut_ctx *c, const int64_t *in, uint64_t n, const int64_t *spl, int ns, int64_t *out,
                                uint64_t *counts_host);  // msd_sort.hip
// f64 bits <-> int64 words in the IEEE total order (an involution; in == out allowed),
// stream-ordered; canon: -0.0 -> +0.0 and NaN -> kF64CanonNaN first (GROUP BY keys)
constexpr uint64_t kF64CanonNaN = 0x7FF8000000000000ull;
nut_status f64_signed_order(nut_ctx *c, const uint64_t *in, uint64_t *out, uint64_t n, bool canon = false);  // sort.hip
nut_status join_matched(nut_ctx *c, const int64_t *bi, uint64_t n, int64_t *out);                   // join.hip
nut_status hash_partition16(nut_ctx *c, const int64_t *keys, uint64_t n, uint64_t kx, int64_t *tmpk,  // aggregate.hip
                            int64_t *tmpr, int64_t *outk, int64_t *outr, std::vector<uint64_t> &counts,
                            const int64_t *rows = nullptr);
// nut_join_i64_into whose pairs carry given row ids: brows[i] for build record i, prows[r]
// for probe record r (NULL: the index) — joins over pushed-down selections (sql_plan.cpp)
nut_status join_i64_into_rows(nut_ctx *c, const int64_t *build, const int64_t *brows, uint64_t nb,
                              const int64_t *probe, const int64_t *prows, uint64_t np, int type, int64_t *probe_idx,
                              int64_t *build_idx, uint64_t cap, uint64_t *npairs);
}  // namespace nut
