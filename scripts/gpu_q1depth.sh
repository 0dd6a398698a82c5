cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 120 scripts/tune/bin/q1_probe > gpurun_out/q1_probe.log 2>&1; rc=$?; cat gpurun_out/q1_probe.log; [ $rc = 0 ] || exit $rc
bash scripts/ab_option.sh 3 agg_depth "1 2" --workload q1 --steps 20 --warmup 3 > gpurun_out/ab_depth.log 2>&1; rc=$?; cat gpurun_out/ab_depth.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload q1 --option agg_depth=2 > gpurun_out/b_depth2.log 2>&1; rc=$?; grep '^{' gpurun_out/b_depth2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'], d['roofline']['copy_floor']['kernel_frac_of_copy'], d['parity'])"; exit $rc
