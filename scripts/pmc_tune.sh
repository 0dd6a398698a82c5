#!/bin/bash
# One rocprofv3 PMC pass (<= 8 SQ counters) over the msd_tune harness; prints every
# dispatch of kernels matching <pattern> in order.
#   scripts/pmc_tune.sh <tag> "<counters>" <pattern> [tune args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
tag=$1; counters=$2; pat=$3; shift 3
out=gpurun_out/pmc_$tag
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --pmc $counters -d "$out" -o pmc --output-format csv -- scripts/tune/bin/msd_tune "$@" > "$out/run.log" 2>&1 || exit $?
python3 - "$out" "$pat" <<'PY'
import collections, csv, glob, sys
d, pat = sys.argv[1], sys.argv[2]
rows = collections.OrderedDict()
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        rows.setdefault(k, {"name": r["Kernel_Name"][:40]})[r["Counter_Name"]] = float(r["Counter_Value"])
for k in sorted(rows):
    v = rows[k]
    print(k, v.pop("name"), " ".join(f"{c}={x:.3e}" for c, x in sorted(v.items())))
PY
