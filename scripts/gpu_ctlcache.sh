# group-by result control words cached between table writes: the group-by / dist / SQL /
# partition GPU suites, then the default bench line
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_exec.py tests/test_gpu_gpart.py tests/test_gpu_dist_native.py tests/test_gpu_groupkeys.py tests/test_gpu_join.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ctl.log 2>&1; rc=$?; tail -3 gpurun_out/t_ctl.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config']['kernel_ms_per_step'], d['roofline']['frac_wall'])" || exit 1; done
