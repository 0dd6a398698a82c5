# group-by PMC passes (SQ counters + HBM bytes) for G = 1000 (on-chip) and G = 1e5 (partitioned)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp NUT_PREBUILT=1
for g in 1000 100000; do
  B="python3 bench.py --workload groupby --groups $g --steps 2 --warmup 1 --no-cpu-baseline"
  bash scripts/pmc_cmd.sh gb${g}_fetch "FETCH_SIZE" $B > /dev/null || exit $?
  bash scripts/pmc_cmd.sh gb${g}_write "WRITE_SIZE" $B > /dev/null || exit $?
  bash scripts/pmc_cmd.sh gb${g}_sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM" $B > /dev/null || exit $?
  bash scripts/pmc_cmd.sh gb${g}_sq2 "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" $B > /dev/null || exit $?
  python3 scripts/pmc_summary.py gpurun_out/gb${g}_pmc.json "group-by G=$g" agg_kernel,gp_scatter gb${g}_fetch gb${g}_write gb${g}_sq gb${g}_sq2
done
