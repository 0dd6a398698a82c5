# group-by / Q1 GPU tests, smoke, the default bench line (Q1, parity + copy floor), a Q1
# kernel trace, and the shared-table group-by occupancy sweep
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_exec.py tests/test_gpu_sql.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "q1 or groupby or Q1 or sql" > gpurun_out/t_q1.log 2>&1; rc=$?; tail -3 gpurun_out/t_q1.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/b_q1.log 2>&1; rc=$?; grep '^{' gpurun_out/b_q1.log > gpurun_out/q1_bench.json; python -c "import json; d=json.load(open('gpurun_out/q1_bench.json')); print(d['ms_per_step'], d['config']['kernel_ms_per_step'], d['roofline']['frac'], d['roofline']['copy_floor']['kernel_frac_of_copy'], d['parity']['ok'])"; [ $rc = 0 ] || exit $rc
mkdir -p gpurun_out/q1trace && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q1trace -o q1 --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/q1trace/bench.log 2>&1 || exit 1
for b in 0 1 2 3; do
  timeout -k 10 200 python bench.py --workload groupby --steps 15 --warmup 3 --no-cpu-baseline --no-copy-floor --option agg_blocks=$b 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('gb agg_blocks=$b', round(d['config']['kernel_ms_per_step'],4))" || exit 1
done
