#!/bin/bash
# A/B of one nut_ctx option on ONE box, variants interleaved per round:
#   scripts/ab_option.sh <rounds> <option> "<v1> <v2> ..." <bench args...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
rounds=$1; opt=$2; vals=$3; shift 3
for round in $(seq 1 "$rounds"); do
  for v in $vals; do
    timeout -k 10 200 python bench.py "$@" --option "$opt=$v" --no-cpu-baseline --no-copy-floor \
      2>/dev/null | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$round', '$opt=$v', 'kernel', round(d['config']['kernel_ms_per_step'], 4), 'step', round(d['ms_per_step'], 4), flush=True)" || exit 1
  done
done
