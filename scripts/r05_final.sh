#!/bin/bash
# Round 5 closing evidence, one part per gpurun call (scripts/round_final_part.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/round_final_part.sh r05 "$1"
