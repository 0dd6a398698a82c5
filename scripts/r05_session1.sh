#!/bin/bash
# Round 5 session 1: sort local-kernel attribution, the ordered group-by clamp, Q1 shape probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "120 lt_stamps scripts/tune/bin/local_tune" \
  "100 pmc_lt_a scripts/pmc_bin.sh lt_a 'SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CU_CYCLES' scripts/tune/bin/local_tune_plain 262144 4768 1" \
  "100 pmc_lt_b scripts/pmc_bin.sh lt_b 'SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_SCA' scripts/tune/bin/local_tune_plain 262144 4768 1" \
  "300 gorder python -u -m pytest tests/test_gpu_gorder.py -x -q --timeout 200 --timeout-method thread" \
  "200 bench_q1 python bench.py --steps 10 --warmup 2"
