#!/bin/bash
# Round 5 session 25: the match-fed write-out with 32-bit ranks (126 VGPRs: two workgroups
# per CU): join tests, the join line twice and a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/join25
scripts/gpu_session.sh \
  "400 t_join python -u -m pytest tests/test_gpu_join.py -q --timeout 200 --timeout-method thread" \
  "200 join_a python bench.py --workload join --no-cpu-baseline" \
  "200 join_b python bench.py --workload join --no-cpu-baseline" \
  "300 trace_join rocprofv3 --kernel-trace --stats -d gpurun_out/join25/trace -o trace -- python bench.py --workload join --steps 5 --warmup 1 --no-cpu-baseline"
