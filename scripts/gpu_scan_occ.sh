# occupancy sweeps of the expression scan (select kernel) and the expression-mode Q12 group-by
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
for r in 1 2; do
for b in 0 1 2 3 4; do
  timeout -k 10 200 python bench.py --workload scanexpr --steps 30 --warmup 3 --no-cpu-baseline --no-copy-floor --option sel_blocks=$b 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r scanexpr sel_blocks=$b', round(d['config']['kernel_ms_per_step'],4))" || exit 1
done
for b in 0 1 2 3; do
  timeout -k 10 200 python bench.py --workload q12expr --steps 15 --warmup 3 --no-cpu-baseline --no-copy-floor --option agg_blocks=$b 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r q12expr agg_blocks=$b', round(d['config']['kernel_ms_per_step'],4))" || exit 1
done
for b in 0 1 2 4; do
  timeout -k 10 200 python bench.py --workload q12join --steps 15 --warmup 3 --no-cpu-baseline --no-copy-floor --option sel_blocks=$b 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r q12join sel_blocks=$b', round(d['config']['kernel_ms_per_step'],4))" || exit 1
done
done
