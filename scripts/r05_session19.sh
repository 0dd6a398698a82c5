#!/bin/bash
# Round 5 session 19: the two-pass join with its 512x16 write-out: tests, bench, trace; and
# whether the 256x8 ordered tile is slow in the one-pass kernel too (diagnostic).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/join19
scripts/gpu_session.sh \
  "400 t_join python -u -m pytest tests/test_gpu_join.py -q --timeout 200 --timeout-method thread" \
  "300 bench_join python bench.py --workload join" \
  "200 join_onepass_cfg1 python bench.py --workload join --no-cpu-baseline --steps 3 --warmup 1 --option join_match=0 --option join_probe_cfg=1" \
  "300 trace_join rocprofv3 --kernel-trace --stats -d gpurun_out/join19/trace -o trace -- python bench.py --workload join --steps 5 --warmup 1 --no-cpu-baseline"
