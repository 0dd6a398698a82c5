#!/bin/bash
# A/B comparison of library builds on ONE box (box-to-box variance of MI355X boards was
# measured at ~12 % for Q1, so cross-call numbers cannot rank variants):
#   scripts/ab_bench.sh <dir with lib*.so> <rounds> <workload> [<workload> ...]
# Each variant runs every workload, alternating, for <rounds> rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
dir=$1; rounds=$2; shift 2
for round in $(seq 1 "$rounds"); do
  for lib in "$dir"/lib*.so; do
    v=$(basename "$lib" .so)
    for w in "$@"; do
      NUTEXEC_LIB=$(realpath "$lib") timeout -k 10 120 python bench.py --workload "$w" --steps 10 --warmup 2 \
        --no-cpu-baseline 2>/dev/null | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$round', '$v', '$w', round(d['config']['kernel_ms_per_step'], 4), flush=True)" || exit 1
    done
  done
done
