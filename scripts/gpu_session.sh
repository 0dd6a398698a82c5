#!/bin/bash
# Run GPU steps in order on the gpurun box; each step has its own time limit.
# Stops at the first step that faults, aborts, segfaults or times out (exit >= 2
# except pytest's "tests failed" = 1), so nothing else touches a sick GPU.
#   scripts/gpu_session.sh "<limit_s> <name> <command...>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  limit=${spec%% *}; rest=${spec#* }; name=${rest%% *}; cmd=${rest#* }
  echo "=== [$name] limit ${limit}s: $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $name ended with $rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
