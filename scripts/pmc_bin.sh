#!/bin/bash
# One SQ PMC pass (<= 8 SQ counters) over a harness binary, summarised per kernel.
#   scripts/pmc_bin.sh <tag> "<counters>" <binary> [args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
tag=$1; shift
counters=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --pmc $counters -d "$out" -o pmc --output-format csv -- "$@" > "$out/run.log" 2>&1 || exit $?
python3 - "$out" <<'PY'
import collections, csv, glob, sys
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
