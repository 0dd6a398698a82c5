#!/bin/bash
# One GPU iteration on a workload: parity tests (-k filter), bench line, kernel trace.
#   scripts/wl_iter.sh <workload> <pytest -k expression> [extra bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
wl=$1; kx=$2; shift 2
mkdir -p gpurun_out
if [ -n "$kx" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -k "$kx" -q --timeout 200 --timeout-method thread > gpurun_out/${wl}_tests.log 2>&1
  echo "tests rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/${wl}_tests.log | tail -5
fi
timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/bench_${wl}.log 2>&1 || { tail -5 gpurun_out/bench_${wl}.log; exit 1; }
python - "$wl" <<'PY'
import json, sys; l=[x for x in open(f"gpurun_out/bench_{sys.argv[1]}.log") if x.startswith("{")][-1]; d=json.loads(l)
print("bench", sys.argv[1], "ms/step", round(d["ms_per_step"],4), "kernel ms", round(d["config"]["kernel_ms_per_step"],4), "frac", round(d["roofline"]["frac"] or 0,3), "value %.3g" % d["value"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${wl} -o ${wl} --output-format csv -- python3 bench.py --workload $wl --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/prof_${wl}.log 2>&1 || exit 1
python - "$wl" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(f"gpurun_out/prof_{sys.argv[1]}/{sys.argv[1]}_kernel_stats.csv")))[:8]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e6, 4))
PY
