# read-floor vs workgroups per CU (q1_probe), then the library's Q1 / G = 1000 group-by
# and the copy-floor probe at 1..8 workgroups per CU, interleaved on one box
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 120 scripts/tune/bin/q1_probe > gpurun_out/q1_probe.log 2>&1; rc=$?; cat gpurun_out/q1_probe.log; [ $rc = 0 ] || exit $rc
bash scripts/ab_option.sh 3 agg_blocks "0 1" --workload q1 --steps 20 --warmup 3 > gpurun_out/ab_blocks_q1.log 2>&1; rc=$?; cat gpurun_out/ab_blocks_q1.log; [ $rc = 0 ] || exit $rc
bash scripts/ab_option.sh 2 agg_blocks "0 1 2 4" --workload groupby --groups 1000 --steps 20 --warmup 3 > gpurun_out/ab_blocks_gb.log 2>&1; rc=$?; cat gpurun_out/ab_blocks_gb.log; [ $rc = 0 ] || exit $rc
for b in 1 2 4 8; do
  timeout -k 10 300 python bench.py --workload q1 --steps 5 --warmup 2 --no-cpu-baseline --option stream_blocks=$b 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('stream_blocks=$b', d['roofline']['copy_floor']['ms'])" || exit 1
done
