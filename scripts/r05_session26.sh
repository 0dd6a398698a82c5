#!/bin/bash
# Round 5 session 26: the match walks' shape (NUT_OPT_JOIN_ANY_CFG: 0 = 256x4, 1 = 512x8,
# 2 = 256x8, 3 = 512x4), interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "200 m0 python bench.py --workload join --no-cpu-baseline" \
  "200 m2 python bench.py --workload join --no-cpu-baseline --option join_any_cfg=2" \
  "200 m1 python bench.py --workload join --no-cpu-baseline --option join_any_cfg=1" \
  "200 m3 python bench.py --workload join --no-cpu-baseline --option join_any_cfg=3" \
  "200 m0b python bench.py --workload join --no-cpu-baseline" \
  "200 m2b python bench.py --workload join --no-cpu-baseline --option join_any_cfg=2"
