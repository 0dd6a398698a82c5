# the multi-GPU bench path at P = 1 (RCCL through nut_dist_create_rank): --dist without
# torchrun, and torchrun with one rank, for q1 / groupby / sort / filter
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
for w in q1 "groupby --groups 1000" sort filter; do
  timeout -k 10 300 python bench.py --dist --workload $w --steps 5 --warmup 2 > gpurun_out/dist.log 2>&1 || { tail -5 gpurun_out/dist.log; exit 1; }
  grep '^{' gpurun_out/dist.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dist', d['config']['workload'], round(d['ms_per_step'],3), d['config'].get('dist',{}).get('nranks'), d['roofline']['frac'])"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/trun.log 2>&1 || { tail -5 gpurun_out/trun.log; exit 1; }
grep '^{' gpurun_out/trun.log | cut -c1-300
