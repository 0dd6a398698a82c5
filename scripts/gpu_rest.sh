# the GPU suites not run since the control-word cache: SQL, typed tables, projections, ORDER BY, probe, smoke
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_sql.py tests/test_gpu_table.py tests/test_gpu_projections.py tests/test_gpu_order_by.py tests/test_gpu_probe.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_rest.log 2>&1; rc=$?; tail -3 gpurun_out/t_rest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
