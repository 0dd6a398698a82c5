# expression-mode (JIT) private-accumulator kernels: Q12 shape occupancy sweep; then the
# expression / SQL GPU tests at the new default
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
for r in 1 2; do
for cfg in "256 8" "0 0" "128 3" "128 4"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --workload q12expr --steps 15 --warmup 3 --no-cpu-baseline --no-copy-floor --option priv_bd=$1 --option priv_blocks=$2 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r q12expr bd=$1 bpc=$2', round(d['config']['kernel_ms_per_step'],4), d['config'].get('groupby_path'))" || exit 1
done; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_expr.py tests/test_gpu_groupkeys.py tests/test_gpu_sql.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_expr.log 2>&1; rc=$?; tail -3 gpurun_out/t_expr.log; exit $rc
