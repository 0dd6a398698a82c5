# the round-end checks the driver runs, in one call: every -m gpu test, smoke(), the default bench line
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
tail -4 gpurun_out/t_all.log
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
grep '^{' gpurun_out/bench_default.log | tail -1 | cut -c1-400
