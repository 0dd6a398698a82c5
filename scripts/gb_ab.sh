# large-G group-by A/B: the scatter variant sweep, then the G = 1e5 / 1e7 bench lines
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 240 ./scripts/tune/bin/gp_tune > gpurun_out/gp_tune.log 2>&1 || exit $?
cat gpurun_out/gp_tune.log
for g in 100000 10000000; do
  timeout -k 10 300 python3 bench.py --workload groupby --groups $g --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/gb_$g.log 2>&1 || exit $?
  tail -1 gpurun_out/gb_$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($g, d['ms_per_step'], d.get('kernel_ms_per_step'), d['roofline']['frac'], d.get('parity'))"
done
