#!/bin/bash
# Round 5 session 13: heavy pass with host-built cuckoo lookups.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "200 hk_tune scripts/tune/bin/hk_tune" \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread" \
  "300 bench_g1e7_skew python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 prof_g1e7_skew rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g1e7_skew -o skew -- python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "500 t_full python -u -m pytest tests/test_gpu_fullsize.py -q -k 'ordered_to_host' --timeout 400 --timeout-method thread"
