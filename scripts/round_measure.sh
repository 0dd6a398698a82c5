#!/bin/bash
# Round evidence for one workload: kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE
# PMC passes (scripts/round_profile.sh), then the default bench line with its CPU baseline
# and parity check.  Results under gpurun_out/<round>/<name>/.
#   NUT_COMMIT=<sha> scripts/round_measure.sh <round> <name> [pmc|trace] [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
round=$1; name=$2; what=$3; shift 3
out=gpurun_out/$round/$name
mkdir -p "$out"
if [ "$what" = pmc ]; then
  scripts/round_profile.sh "${round}_$name" "$@" > "$out/profile.log" 2>&1 || { tail -5 "$out/profile.log"; exit 1; }
  cp gpurun_out/prof_${round}_$name/summary.json "$out/" && cp gpurun_out/prof_${round}_$name/pmc_*.json "$out/" \
    && cp gpurun_out/prof_${round}_$name/trace/trace_kernel_stats.csv "$out/kernel_stats.csv" || exit 1
else
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace --output-format csv -- \
    python3 bench.py "$@" --no-cpu-baseline > "$out/trace.log" 2>&1 || { tail -5 "$out/trace.log"; exit 1; }
  cp "$out/trace/trace_kernel_stats.csv" "$out/kernel_stats.csv" || exit 1
fi
timeout -k 10 300 python3 bench.py "$@" > "$out/bench.log" 2>&1 || { tail -5 "$out/bench.log"; exit 1; }
grep '^{' "$out/bench.log" | tail -1 > "$out/bench.json"
python3 - "$out/bench.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
r = d["roofline"]
print(sys.argv[2], "ms/step %.3f" % d["ms_per_step"], "kernel %.3f" % d["config"]["kernel_ms_per_step"],
      "frac %.3f" % (r["frac"] or 0), "value %.3g" % d["value"], "parity", (d.get("parity") or {}).get("ok"),
      "cpu %.3g" % (d.get("cpu_baseline") or {}).get("value", 0))
PY
