cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
bash scripts/ab_lib.sh "tests/test_gpu_gorder.py" --workload groupby --groups 10000000 || exit $?
NUTEXEC_LIB=$PWD/nutdb_amd/libnutexec_var.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prio_trace -o trace --output-format csv -- python3 bench.py --workload groupby --groups 10000000 --no-cpu-baseline --steps 4 > gpurun_out/prio_trace.log 2>&1 || exit $?
