#!/bin/bash
# Round 5 session 18: the two-pass ordered join's write-out tile shape (NUT_OPT_JOIN_PROBE_CFG
# picks the ordered pass's tile: 0 = 512x8, 1 = 256x8, 2 = 256x16, 3 = 512x16, 4 = 256x4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "200 join_cfg0 python bench.py --workload join --no-cpu-baseline" \
  "200 join_cfg3 python bench.py --workload join --no-cpu-baseline --option join_probe_cfg=3" \
  "200 join_cfg2 python bench.py --workload join --no-cpu-baseline --option join_probe_cfg=2" \
  "200 join_cfg1 python bench.py --workload join --no-cpu-baseline --option join_probe_cfg=1" \
  "200 join_cfg0b python bench.py --workload join --no-cpu-baseline"
