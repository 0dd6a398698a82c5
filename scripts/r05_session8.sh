#!/bin/bash
# Round 5 session 8: fixture-9 localisation, the heavy pass's counters, sample counts by hash
# table, arena rows partitioned; gorder tests, Zipf / uniform lines, full-size sort test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="python bench.py --workload groupby --groups 10000000 --skew --steps 2 --warmup 1 --no-cpu-baseline --no-copy-floor"
scripts/gpu_session.sh \
  "200 q22dbg python -u scripts/diag/q22_debug.py" \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread" \
  "300 bench_g1e7_skew python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "300 bench_g1e7 python bench.py --workload groupby --groups 10000000 --steps 5 --warmup 2 --no-cpu-baseline" \
  "150 pmc_hk_a scripts/pmc_cmd.sh hk_a 'SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS' $B" \
  "150 pmc_hk_b scripts/pmc_cmd.sh hk_b 'SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR' $B" \
  "500 t_full python -u -m pytest tests/test_gpu_fullsize.py -q -k 'ordered_to_host or sort' --timeout 400 --timeout-method thread"
