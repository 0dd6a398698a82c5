#!/bin/bash
# Probe tile-shape sweep of the hash join (join.hip NUT_HJ_CFG), one bench line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for c in "$@"; do
  NUT_HJ_CFG=$c timeout -k 10 200 python bench.py --workload join --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/join_cfg$c.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['config']['kernel_ms_per_step'])" gpurun_out/join_cfg$c.log $c
done
