# same-box A/B of variant libraries (nutdb_amd/libnutexec_<v>.so) on the ordered large-G
# group-by, uniform and Zipf-like keys:  scripts/tune/ab_gb1e7.sh var [var2 ...]
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
for v in "$@"; do
  NUTEXEC_LIB=$PWD/nutdb_amd/libnutexec_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gorder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests_$v.log 2>&1 || { tail -5 gpurun_out/ab_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/ab_tests_$v.log)"
done
for r in 1 2; do
  for skew in "" "--skew"; do
    for v in base "$@"; do
      if [ $v = base ]; then L=$PWD/nutdb_amd/libnutexec.so; else L=$PWD/nutdb_amd/libnutexec_$v.so; fi
      NUTEXEC_LIB=$L timeout -k 10 200 python3 bench.py --workload groupby --groups 10000000 $skew --no-cpu-baseline > gpurun_out/abg_${v}_$r.log 2>&1 || exit $?
      tail -1 gpurun_out/abg_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${skew:-uniform} $v', round(d['ms_per_step'],3), 'parity', (d.get('parity') or {}).get('ok'))"
    done
  done
done
