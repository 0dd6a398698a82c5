#!/bin/bash
# Round 5 session 15: exact per-cell layout behind the heavy-key pass (no arenas): gorder
# tests, the Zipf G = 1e7 line vs the capped layout (gb_heavy = 2), uniform control, the
# full-size skew test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread" \
  "300 bench_zipf_exact python bench.py --workload groupby --groups 10000000 --skew" \
  "300 bench_zipf_capped python bench.py --workload groupby --groups 10000000 --skew --option gb_heavy=2" \
  "300 bench_zipf_exact2 python bench.py --workload groupby --groups 10000000 --skew" \
  "300 bench_g1e7 python bench.py --workload groupby --groups 10000000" \
  "500 t_full python -u -m pytest tests/test_gpu_fullsize.py -q -k ordered_to_host --timeout 400 --timeout-method thread"
