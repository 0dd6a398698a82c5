#!/bin/bash
# Kernel timeline of one large-G group-by step: scripts/gb_trace.sh <groups>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
g=$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gb$g -o gb --output-format csv -- python3 bench.py --workload groupby --groups $g --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_gb$g.log 2>&1 || exit 1
grep '^{' gpurun_out/prof_gb$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('G', $g, 'ms/step', round(d['ms_per_step'],3), 'kernel ms', round(d['config']['kernel_ms_per_step'],3))"
python3 - "$g" <<'PY'
import csv, sys
g = sys.argv[1]
rows = sorted(csv.DictReader(open(f"gpurun_out/prof_gb{g}/gb_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
# the last step: from the last agg_kernel launch in spill mode back... print the last 40 dispatches
t0 = None
for r in rows[-40:]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 is None: t0 = st; prev = st
    print(f'{(st-t0)/1e6:8.3f} gap {(st-prev)/1e6:6.3f} dur {(en-st)/1e6:7.3f} {r["Kernel_Name"][:60]}')
    prev = en
PY
