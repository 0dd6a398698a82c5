# SQ counters of the Q1 kernel (one pass of 8): where its wave cycles go
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1
bash scripts/pmc_sq.sh q1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" --workload q1 --steps 3 --warmup 1 > gpurun_out/sq_q1.txt 2>&1; rc=$?; cat gpurun_out/sq_q1.txt; [ $rc = 0 ] || exit $rc
bash scripts/pmc_sq.sh gb "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" --workload groupby --steps 3 --warmup 1 > gpurun_out/sq_gb.txt 2>&1; rc=$?; cat gpurun_out/sq_gb.txt; exit $rc
