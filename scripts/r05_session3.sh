#!/bin/bash
# Round 5 session 3: local-sort variant sweep (restructured kernel), ordered group-by parity
# with the decline reason, the G = 1e7 ordered bench line (uniform and Zipf-like keys).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "150 lt_sweep scripts/tune/bin/local_tune_plain" \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread" \
  "300 bench_g1e7 python bench.py --workload groupby --groups 10000000 --steps 5 --warmup 2" \
  "300 bench_g1e7_skew python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2"
