#!/bin/bash
# Round 6: the 0.5-s join cliff — one traced run of the 512 x 4 match
# walks (join_any_cfg = 3) next to the default, then one SQ + one TCP counter pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/cliff
J="python bench.py --workload join --steps 3 --warmup 1 --no-cpu-baseline --no-copy-floor"
scripts/gpu_session.sh \
  "200 cliff_def $J" \
  "200 cliff_m3 $J --option join_any_cfg=3" \
  "300 cliff_trace rocprofv3 --kernel-trace --stats -d gpurun_out/cliff/trace -o trace --output-format csv -- $J --option join_any_cfg=3" \
  "200 cliff_m3b $J --option join_any_cfg=3" \
  "120 cliff_sq timeout -s KILL 110 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY -d gpurun_out/cliff/sq -o sq --output-format csv -- $J --option join_any_cfg=3" \
  "60 avail rocprofv3 --list-avail"
