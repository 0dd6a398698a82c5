# Sort (config 5) evidence: kernel trace + PMC (HBM bytes; VALU / LDS / bank conflicts) of the bench line
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp NUT_PREBUILT=1
if [ "$1" != "pmc" ]; then
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sort -o run --output-format csv -- python3 bench.py --workload sort --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_sort.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_sort/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print('  %-70s %5s %10.1f us' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
PY
tail -1 gpurun_out/prof_sort.log | cut -c1-300
fi
B="python3 bench.py --workload sort --steps 2 --warmup 1 --no-cpu-baseline"
bash scripts/pmc_cmd.sh sort_fetch "FETCH_SIZE" $B || exit $?
bash scripts/pmc_cmd.sh sort_write "WRITE_SIZE" $B || exit $?
bash scripts/pmc_cmd.sh sort_sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM" $B || exit $?
