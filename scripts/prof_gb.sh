cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp NUT_PREBUILT=1
for g in 100000 10000000; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gb$g -o run --output-format csv -- python3 bench.py --workload groupby --groups $g --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_gb$g.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob
for g in (100000, 10000000):
    f = glob.glob(f'gpurun_out/prof_gb{g}/**/*kernel_stats.csv', recursive=True)[0]
    print(g, f)
    for r in csv.DictReader(open(f)):
        print('  %-70s %5s %10.1f us' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
PY
tail -1 gpurun_out/prof_gb100000.log | cut -c1-400; tail -1 gpurun_out/prof_gb10000000.log | cut -c1-400
