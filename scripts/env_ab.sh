#!/bin/bash
# A/B of one library build under two values of an environment switch, alternating on ONE box:
#   scripts/env_ab.sh <VAR> "<values>" <rounds> <bench args...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
var=$1; vals=$2; rounds=$3; shift 3
for round in $(seq 1 "$rounds"); do
  for v in $vals; do
    env "$var=$v" timeout -k 10 200 python bench.py "$@" --steps 8 --warmup 2 --no-cpu-baseline 2>/dev/null | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$round', '$var=$v', '$*', 'kernel', round(d['config']['kernel_ms_per_step'], 3), 'step', round(d['ms_per_step'], 3), flush=True)" || exit 1
  done
done
