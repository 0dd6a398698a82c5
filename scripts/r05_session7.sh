#!/bin/bash
# Round 5 session 7: fixture-9 localisation, heavy pass with batched probes + value-count
# templates, wider level-1 regions under heavy keys, arena rows via a copy, the clamp folded
# into the aggregation; gorder / substring / group-by tests, Zipf + uniform lines and traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "200 q22dbg python -u scripts/diag/q22_debug.py" \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread" \
  "400 t_gb python -u -m pytest tests/test_gpu_exec.py -q -k 'groupby or partition' --timeout 200 --timeout-method thread" \
  "300 bench_g1e7_skew python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 prof_g1e7_skew rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g1e7_skew -o skew -- python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "300 bench_g1e7 python bench.py --workload groupby --groups 10000000 --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 prof_g1e7 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g1e7 -o g1e7 -- python bench.py --workload groupby --groups 10000000 --steps 5 --warmup 2 --no-cpu-baseline" \
  "500 t_full python -u -m pytest tests/test_gpu_fullsize.py -q -k 'ordered_to_host or config3' --timeout 400 --timeout-method thread"
