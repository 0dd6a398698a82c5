#!/bin/bash
# Evidence for profiles/: rocprofv3 kernel-trace stats of the default bench command and
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the same command, summarised into
# gpurun_out/prof_round/{summary.json,pmc_<workload>.json}.
#   scripts/round_profile.sh <round-tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
args=("$@" --no-cpu-baseline)
set -o pipefail
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace --output-format csv -- python3 bench.py "${args[@]}" > "$out/trace.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o fetch --output-format csv -- python3 bench.py "${args[@]}" --no-copy-floor > "$out/fetch.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o write --output-format csv -- python3 bench.py "${args[@]}" --no-copy-floor > "$out/write.log" 2>&1 || exit $?
python3 scripts/pmc_traffic.py "$out" "${args[@]}"
