#!/bin/bash
# Round 5: attribution of the sort's local kernel (per-phase s_memtime stamps + SQ PMC passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "120 lt_stamps scripts/tune/bin/local_tune" \
  "100 pmc_lt_a scripts/pmc_bin.sh lt_a 'SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CU_CYCLES' scripts/tune/bin/local_tune_plain 262144 4768 1" \
  "100 pmc_lt_b scripts/pmc_bin.sh lt_b 'SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_SCA' scripts/tune/bin/local_tune_plain 262144 4768 1"
