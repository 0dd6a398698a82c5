#!/bin/bash
# Round 5 session 5: heavy-key pass of the ordered group-by (gorder tests, Zipf / uniform
# G = 1e7 lines, the 1e9-row Zipf parity test), substring / fixture 9, UNION ALL, subquery
# regressions, and the G = 1e5 level-0 digit width A/B (7 vs 6 bits).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread" \
  "300 t_sql python -u -m pytest tests/test_gpu_substring.py tests/test_gpu_union.py tests/test_gpu_subquery.py tests/test_gpu_derived.py -q --timeout 200 --timeout-method thread" \
  "300 bench_g1e7_skew python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "300 bench_g1e7 python bench.py --workload groupby --groups 10000000 --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 prof_g1e7_skew rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g1e7_skew -o skew -- python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 bench_g1e5_l7 python bench.py --workload groupby --groups 100000 --steps 10 --warmup 2 --no-cpu-baseline" \
  "200 bench_g1e5_l6 python bench.py --workload groupby --groups 100000 --steps 10 --warmup 2 --no-cpu-baseline --option gb_l0_bits=6" \
  "200 bench_g1e5_l7b python bench.py --workload groupby --groups 100000 --steps 10 --warmup 2 --no-cpu-baseline" \
  "200 bench_g1e5_l6b python bench.py --workload groupby --groups 100000 --steps 10 --warmup 2 --no-cpu-baseline --option gb_l0_bits=6" \
  "500 t_full python -u -m pytest tests/test_gpu_fullsize.py -q -k ordered_to_host --timeout 400 --timeout-method thread"
