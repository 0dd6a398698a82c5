#!/bin/bash
# Round 5 session 17: the ordered join in two passes (match array + ordered write-out):
# join tests, then the config (f)4 join line with the option on / off / on, and a trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/join17
scripts/gpu_session.sh \
  "400 t_join python -u -m pytest tests/test_gpu_join.py -q --timeout 200 --timeout-method thread" \
  "300 bench_join_two python bench.py --workload join" \
  "300 bench_join_one python bench.py --workload join --option join_match=0" \
  "300 bench_join_two2 python bench.py --workload join" \
  "300 trace_join rocprofv3 --kernel-trace --stats -d gpurun_out/join17/trace -o trace -- python bench.py --workload join --steps 5 --warmup 1 --no-cpu-baseline"
