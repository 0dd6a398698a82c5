# Q1 kernel occupancy: threads per workgroup x workgroups per CU (interleaved, one box)
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
for r in 1 2; do
for cfg in "0 0" "128 3" "128 2" "192 2" "128 4" "256 1" "192 1"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --workload q1 --steps 15 --warmup 3 --no-cpu-baseline --no-copy-floor --option priv_bd=$1 --option priv_blocks=$2 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r bd=$1 bpc=$2', round(d['config']['kernel_ms_per_step'],4))" || exit 1
done; done
