#!/bin/bash
# Round 5 session 27: persistent region build with the next region's records prefetched:
# join tests, a trace, the join and Q12 join lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/join27
scripts/gpu_session.sh \
  "400 t_join python -u -m pytest tests/test_gpu_join.py -q --timeout 200 --timeout-method thread" \
  "300 trace_join rocprofv3 --kernel-trace --stats -d gpurun_out/join27/trace -o trace --output-format csv -- python bench.py --workload join --steps 5 --warmup 1 --no-cpu-baseline" \
  "200 join_a python bench.py --workload join --no-cpu-baseline" \
  "200 q12join python bench.py --workload q12join --no-cpu-baseline"
