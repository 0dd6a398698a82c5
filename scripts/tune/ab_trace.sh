# kernel stats of the product library and the variant library on one bench workload
#   scripts/tune/ab_trace.sh <bench args...>
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1 TMPDIR=/tmp
for v in base var; do
  if [ $v = var ]; then L=$PWD/nutdb_amd/libnutexec_var.so; else L=$PWD/nutdb_amd/libnutexec.so; fi
  NUTEXEC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abt_$v -o trace --output-format csv -- python3 bench.py "$@" --no-cpu-baseline --steps 4 > gpurun_out/abt_$v.log 2>&1 || exit $?
  python3 - gpurun_out/abt_$v/trace_kernel_stats.csv $v <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:6]:
    print(sys.argv[2], x['Name'][:70], x['Calls'], round(float(x['AverageNs']) / 1e6, 3))
PY
done
