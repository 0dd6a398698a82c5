#!/bin/bash
# One GPU iteration on the sort: parity tests, bench line, kernel trace, local-sort harness.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -k "sort or order or fullsize" -q --timeout 200 --timeout-method thread > gpurun_out/sort_tests.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed" gpurun_out/sort_tests.log | tail -3
timeout -k 10 300 python bench.py --workload sort --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_sort.log 2>&1 || exit 1
python - <<'PY'
import json; l=[x for x in open("gpurun_out/bench_sort.log") if x.startswith("{")][-1]; d=json.loads(l)
print("bench sort ms/step", round(d["ms_per_step"],3), "kernel ms", round(d["config"]["kernel_ms_per_step"],3))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sort -o sort --output-format csv -- python3 bench.py --workload sort --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_sort.log 2>&1 || exit 1
python - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_sort/sort_kernel_stats.csv")):
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e6, 3))
PY
if [ -n "$1" ]; then timeout -k 10 200 scripts/tune/bin/msd_tune 1250000000 "$1" 2>&1 | grep local; fi
