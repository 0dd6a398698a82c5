# Large-G group-by evidence at HEAD: bench lines with full-size parity (indexed oracle) and
# a kernel trace of each
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp NUT_PREBUILT=1
for g in 100000 10000000; do
  timeout -k 10 300 python3 bench.py --workload groupby --groups $g --steps 10 --warmup 2 > gpurun_out/gbev_$g.log 2>&1 || exit $?
  grep '^{' gpurun_out/gbev_$g.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($g, round(d['ms_per_step'],3), round(d['config']['kernel_ms_per_step'],3), round(d['roofline']['frac'],4), d['config']['groupby_path'], d.get('parity'))"
done
bash scripts/prof_gb.sh
