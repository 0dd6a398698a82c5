cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_sql.py tests/test_gpu_table.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sql.log 2>&1; rc=$?; tail -15 gpurun_out/t_sql.log; [ $rc = 0 ] || exit $rc
bash scripts/gpu_scan_occ.sh
