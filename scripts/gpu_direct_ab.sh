# group-by GPU tests on the direct-map build, then Q1 / G = 1000 A/B of the hash-only
# (libA) and direct-map (libB) builds on one box, then the Q1 bench line with parity
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_exec.py tests/test_gpu_sql.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gb.log 2>&1; rc=$?; tail -3 gpurun_out/t_gb.log; [ $rc = 0 ] || exit $rc
bash scripts/ab_bench.sh scripts/tune/bin/ab 3 q1 > gpurun_out/ab_direct.log 2>&1; rc=$?; cat gpurun_out/ab_direct.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/b_q1.log 2>&1; rc=$?; grep '^{' gpurun_out/b_q1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'], d['roofline']['copy_floor'], d['parity']['ok'])"; exit $rc
