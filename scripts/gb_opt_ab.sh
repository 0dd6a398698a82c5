# same-box A/B of one nut_ctx option on the large-G group-by bench lines
#   scripts/gb_opt_ab.sh <option> <value>...
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
opt=$1; shift
for g in 100000 10000000; do
  for v in "$@" "$@"; do
    timeout -k 10 300 python3 bench.py --workload groupby --groups $g --steps 10 --warmup 2 --no-cpu-baseline --option $opt=$v > gpurun_out/gbab_${g}_$v.log 2>&1 || exit $?
    tail -1 gpurun_out/gbab_${g}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('G=$g $opt=$v', round(d['ms_per_step'],3), 'kernels', round(d['config']['kernel_ms_per_step'],3))"
  done
done
