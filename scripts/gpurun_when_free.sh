#!/bin/bash
# Submit one gpurun call, resubmitting only while the pool has no free box (exit 3: nothing
# ran, nothing charged) — never after a run that started.  Usage:
#   scripts/gpurun_when_free.sh <log> <timeout_s> <command>
log=$1; to=$2; shift 2
for attempt in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  echo "[attempt $attempt rc=$rc]" >> "$log"
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
exit 3
