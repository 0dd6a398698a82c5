#!/bin/bash
# Round 5 session 14: the two-value heavy-pass test, G = 1e5 with the faster CPU baseline,
# the RCCL P = 1 bench path and the dist tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread" \
  "300 bench_g1e5 python bench.py --workload groupby --groups 100000" \
  "300 bench_q1_dist python bench.py --dist --steps 5 --warmup 1" \
  "500 t_dist python -u -m pytest tests/test_gpu_dist_native.py -q --timeout 300 --timeout-method thread"
