#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes for one bench workload.
#   scripts/profile.sh <tag> <bench args...>
# Writes gpurun_out/prof_<tag>/... ; each pass has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv -- python3 bench.py "${BENCH_ARGS[@]}" > "$out/$name.log" 2>&1
  local rc=$?
  echo "[profile $tag/$name] rc=$rc"
  return $rc
}
BENCH_ARGS=("$@" --no-cpu-baseline)
run trace --kernel-trace --stats || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT || exit $?
exit 0
