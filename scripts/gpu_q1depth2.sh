# Q1: workgroups per CU x prefetch depth (interleaved, one box); copy-floor probe workgroups
# per CU for the filter's 2:1 read:write stream
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
bash scripts/ab_option.sh 3 agg_blocks "0 1" --workload q1 --steps 20 --warmup 3 --option agg_depth=2 > gpurun_out/ab_q1_d2.log 2>&1; rc=$?; cat gpurun_out/ab_q1_d2.log; [ $rc = 0 ] || exit $rc
bash scripts/ab_option.sh 2 agg_depth "1" --workload q1 --steps 20 --warmup 3 > gpurun_out/ab_q1_d1.log 2>&1; rc=$?; cat gpurun_out/ab_q1_d1.log; [ $rc = 0 ] || exit $rc
for w in filter groupby; do for b in 1 2 4 8; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --option stream_blocks=$b 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w stream_blocks=$b', d['roofline']['copy_floor']['ms'], d['config']['kernel_ms_per_step'])" || exit 1
done; done
