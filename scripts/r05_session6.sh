#!/bin/bash
# Round 5 session 6: heavy-key pass as per-workgroup chunks (no cursor atomics) with its
# groups inserted into their partitions on the device; gorder / substring / fullsize tests;
# Zipf and uniform G = 1e7 lines with kernel traces; the sort's local-kernel attribution.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread" \
  "300 t_sub python -u -m pytest tests/test_gpu_substring.py -q --timeout 200 --timeout-method thread" \
  "300 bench_g1e7_skew python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 prof_g1e7_skew rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g1e7_skew -o skew -- python bench.py --workload groupby --groups 10000000 --skew --steps 5 --warmup 2 --no-cpu-baseline" \
  "300 bench_g1e7 python bench.py --workload groupby --groups 10000000 --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 prof_g1e7 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g1e7 -o g1e7 -- python bench.py --workload groupby --groups 10000000 --steps 5 --warmup 2 --no-cpu-baseline" \
  "200 prof_g1e5 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g1e5 -o g1e5 -- python bench.py --workload groupby --groups 100000 --steps 10 --warmup 2 --no-cpu-baseline" \
  "500 t_full python -u -m pytest tests/test_gpu_fullsize.py -q -k ordered_to_host --timeout 400 --timeout-method thread" \
  "120 lt_stamps scripts/tune/bin/local_tune 262144 4768" \
  "100 pmc_lt_a scripts/pmc_bin.sh lt_a 'SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CU_CYCLES' scripts/tune/bin/local_tune_plain 262144 4768 1" \
  "100 pmc_lt_b scripts/pmc_bin.sh lt_b 'SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU' scripts/tune/bin/local_tune_plain 262144 4768 1"
