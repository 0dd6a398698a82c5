#!/bin/bash
# Round 5 session 4: M sort classes one workgroup per segment (sort tests, bench, kernel
# trace); ordered group-by partitions cut at their first arena run (gorder tests, G = 1e7
# uniform / Zipf lines); UNION ALL on the GPU; partition scatter variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "400 t_sort python -u -m pytest tests/test_gpu_exec.py tests/test_gpu_sort_range.py tests/test_gpu_order_by.py -x -q -k 'sort or order' --timeout 200 --timeout-method thread" \
  "200 bench_sort python bench.py --workload sort --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 prof_sort rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sort -o sort -- python bench.py --workload sort --steps 5 --warmup 2 --no-cpu-baseline" \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread" \
  "300 t_union python -u -m pytest tests/test_gpu_union.py -q --timeout 200 --timeout-method thread" \
  "300 bench_g1e7 python bench.py --workload groupby --groups 10000000 --steps 5 --warmup 2 --no-cpu-baseline" \
  "300 bench_g1e7_skew python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "150 gp_tune scripts/tune/bin/gp_tune"
