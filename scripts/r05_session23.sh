#!/bin/bash
# Round 5 session 23: the ordered path's level 1 at 512-thread scatter workgroups, so the
# previous chunk's aggregation can share the CUs (NUT_OPT_GB_L1_THREADS): parity, then an
# interleaved A/B at G = 1e7, uniform and Zipf-like keys.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "300 t_narrow python -u -m pytest tests/test_gpu_gorder.py -q -k narrow --timeout 200 --timeout-method thread" \
  "200 u1024 python bench.py --workload groupby --groups 10000000 --no-cpu-baseline" \
  "200 u512 python bench.py --workload groupby --groups 10000000 --no-cpu-baseline --option gb_l1_threads=512" \
  "200 z1024 python bench.py --workload groupby --groups 10000000 --skew --no-cpu-baseline" \
  "200 z512 python bench.py --workload groupby --groups 10000000 --skew --no-cpu-baseline --option gb_l1_threads=512" \
  "200 u1024b python bench.py --workload groupby --groups 10000000 --no-cpu-baseline" \
  "200 u512b python bench.py --workload groupby --groups 10000000 --no-cpu-baseline --option gb_l1_threads=512"
