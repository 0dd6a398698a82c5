cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_exec.py tests/test_gpu_sort_range.py tests/test_gpu_fullsize.py tests/test_gpu_sql.py -k "sort or order" -x -q --timeout 300 --timeout-method thread > gpurun_out/t_sort.log 2>&1; rc=$?; tail -3 gpurun_out/t_sort.log; exit $rc
