#!/bin/bash
# Round 5 session 16: G = 1e5 scatter — the product's output layout vs separate allocations
# in the harness, and the product bench on the same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "200 gp_layout scripts/tune/bin/gp_tune 1e9 1e5 layout" \
  "300 bench_g1e5 python bench.py --workload groupby --groups 100000" \
  "200 gp_product scripts/tune/bin/gp_tune 1e9 1e5 product"
