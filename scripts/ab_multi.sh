# same-box A/B of a variant library (nutdb_amd/libnutexec_var.so) on several bench workloads
#   scripts/ab_multi.sh "<tests>" "<bench args 1>" ["<bench args 2>" ...]
# runs the tests with the variant, then each workload var / base / var / base
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
t=$1; shift
NUTEXEC_LIB=$PWD/nutdb_amd/libnutexec_var.so timeout -k 10 400 python -u -m pytest $t -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -5 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
k=0
for w in "$@"; do
  k=$((k + 1))
  for r in 1 2; do
    for v in var base; do
      if [ $v = var ]; then L=$PWD/nutdb_amd/libnutexec_var.so; else L=$PWD/nutdb_amd/libnutexec.so; fi
      NUTEXEC_LIB=$L timeout -k 10 200 python3 bench.py $w --no-cpu-baseline > gpurun_out/abm_${k}_${v}_$r.log 2>&1 || exit $?
      tail -1 gpurun_out/abm_${k}_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', '$v', round(d['ms_per_step'],3), 'kernels', round(d['config'].get('kernel_ms_per_step', 0),3), 'parity', (d.get('parity') or {}).get('ok'))"
    done
  done
done
