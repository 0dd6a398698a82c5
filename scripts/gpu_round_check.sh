# local-sort sweep (window stride / bucket bits; large segments) then the round-end checks
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 scripts/tune/bin/local_tune > gpurun_out/local_tune_ws.log 2>&1 || exit $?
timeout -k 10 120 scripts/tune/bin/local_tune 65536 19073 > gpurun_out/local_tune_large.log 2>&1 || exit $?
bash scripts/full_gpu.sh
