#!/bin/bash
# A/B of library builds on ONE box with explicit bench arguments:
#   scripts/ab_args.sh <dir with lib*.so> <rounds> <bench args...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
dir=$1; rounds=$2; shift 2
for round in $(seq 1 "$rounds"); do
  for lib in "$dir"/lib*.so; do
    v=$(basename "$lib" .so)
    NUTEXEC_LIB=$(realpath "$lib") timeout -k 10 200 python bench.py "$@" --steps 8 --warmup 2 --no-cpu-baseline \
      2>/dev/null | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$round', '$v', '$*', 'kernel', round(d['config']['kernel_ms_per_step'], 3), 'step', round(d['ms_per_step'], 3), flush=True)" || exit 1
  done
done
