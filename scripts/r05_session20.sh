#!/bin/bash
# Round 5 session 20: bucket-aligned join runs (NUT_OPT_JOIN_BUCKET) — parity, then an
# interleaved A/B of the join line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "300 t_join_bucket python -u -m pytest tests/test_gpu_join.py -q -k one_vs_two --timeout 200 --timeout-method thread" \
  "200 join_b0 python bench.py --workload join --no-cpu-baseline" \
  "200 join_b1 python bench.py --workload join --no-cpu-baseline --option join_bucket=1" \
  "200 join_b0b python bench.py --workload join --no-cpu-baseline" \
  "200 join_b1b python bench.py --workload join --no-cpu-baseline --option join_bucket=1" \
  "200 join_any_b0 python bench.py --workload join --no-cpu-baseline --option join_match=0" 
