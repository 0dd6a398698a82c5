#!/bin/bash
# Round 5 session 2: local-sort restructure (single prefetch site) vs HEAD, sort + ordered
# group-by parity, Q1 shape probe, sort bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "120 lt_head scripts/tune/bin/local_tune_head" \
  "120 lt_new scripts/tune/bin/local_tune_plain" \
  "400 t_sort python -u -m pytest tests/test_gpu_exec.py tests/test_gpu_sort_range.py tests/test_gpu_order_by.py -x -q -k 'sort or order' --timeout 200 --timeout-method thread" \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -x -q --timeout 200 --timeout-method thread" \
  "200 bench_sort python bench.py --workload sort --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 bench_q1 python bench.py --steps 10 --warmup 2"
