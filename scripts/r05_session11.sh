#!/bin/bash
# Round 5 session 11: heavy pass with batched probe reads and one kind dispatch per aggregate.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread" \
  "300 bench_g1e7_skew python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 prof_g1e7_skew rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g1e7_skew -o skew -- python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "300 bench_g1e7 python bench.py --workload groupby --groups 10000000 --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 prof_g1e7 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g1e7 -o g1e7 -- python bench.py --workload groupby --groups 10000000 --steps 5 --warmup 2 --no-cpu-baseline"
