cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_probe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_probe.log 2>&1; rc=$?; tail -3 gpurun_out/t_probe.log; [ $rc = 0 ] || exit $rc
for w in "q1" "filter" "groupby --groups 1000" "scanexpr" "sort"; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  grep '^{' gpurun_out/b.log | tail -1 >> gpurun_out/cf_lines.jsonl
  grep '^{' gpurun_out/b.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['config']['workload'], d['ms_per_step'], r['frac'], r['frac_wall'], r['copy_floor'])"
done
