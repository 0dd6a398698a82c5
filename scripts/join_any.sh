#!/bin/bash
# Unordered-probe tile-shape sweep (join.hip NUT_HJ_ANYCFG) on the q12join workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for v in "$@"; do
  NUT_HJ_ANYCFG=$v timeout -k 10 200 python bench.py --workload q12join --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/join_any$v.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" gpurun_out/join_any$v.log $v
done
