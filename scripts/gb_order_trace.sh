cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
for o in 0 1; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_go$o -o go --output-format csv -- python3 bench.py --workload groupby --groups 10000000 --steps 3 --warmup 1 --no-cpu-baseline --no-copy-floor --option gb_ordered=$o > gpurun_out/prof_go$o.log 2>&1 || exit 1
python3 - $o <<'PY'
import csv, sys
o = sys.argv[1]
for r in sorted(csv.DictReader(open(f"gpurun_out/prof_go{o}/go_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"])):
    print(o, r["Name"][:75], r["Calls"], round(float(r["AverageNs"])/1e6, 3), round(float(r["TotalDurationNs"])/1e6/4, 3))
PY
done
