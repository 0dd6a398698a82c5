cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 120 scripts/tune/bin/q1_probe > gpurun_out/q1_probe.log 2>&1; rc=$?; cat gpurun_out/q1_probe.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_exec.py -k filter -x -q --timeout 120 --timeout-method thread > gpurun_out/t_filter.log 2>&1; rc=$?; tail -3 gpurun_out/t_filter.log; [ $rc = 0 ] || exit $rc
bash scripts/ab_option.sh 4 filter_split "0 1" --workload filter --steps 50 --warmup 5 > gpurun_out/ab_split.log 2>&1; rc=$?; cat gpurun_out/ab_split.log; exit $rc
