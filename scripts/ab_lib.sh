# same-box A/B of a variant library (nutdb_amd/libnutexec_var.so) on one bench workload
#   scripts/ab_lib.sh <tests-to-run-with-the-variant> <bench args...>
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
t=$1; shift
NUTEXEC_LIB=$PWD/nutdb_amd/libnutexec_var.so timeout -k 10 300 python -u -m pytest $t -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -5 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in 1 2 3; do
  for v in base var; do
    if [ $v = var ]; then L=$PWD/nutdb_amd/libnutexec_var.so; else L=$PWD/nutdb_amd/libnutexec.so; fi
    NUTEXEC_LIB=$L timeout -k 10 200 python3 bench.py "$@" --no-cpu-baseline > gpurun_out/ab_${v}_$r.log 2>&1 || exit $?
    tail -1 gpurun_out/ab_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],3), 'kernels', round(d['config']['kernel_ms_per_step'],3), 'parity', (d.get('parity') or {}).get('ok'))"
  done
done
