#!/bin/bash
# Round 6 GPU sessions: scripts/r06_session.sh NAME — one named set of steps (each with its own
# time limit, stopping at the first fault / abort / timeout; scripts/gpu_session.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
B="python bench.py --no-cpu-baseline"
case "$1" in
  s2)
    mkdir -p gpurun_out/g1000
    scripts/gpu_session.sh \
      "600 t_s2 $T tests/test_gpu_f64_scan.py tests/test_gpu_dist_native.py tests/test_gpu_gorder.py tests/test_gpu_exec.py" \
      "300 frag scripts/tune/bin/frag_probe 0.8" \
      "200 g1000_a $B --workload groupby --groups 1000" \
      "200 g1000_b1 $B --workload groupby --groups 1000 --option agg_blocks=1" \
      "200 g1000_b $B --workload groupby --groups 1000" \
      "300 g1000_trace rocprofv3 --kernel-trace --stats -d gpurun_out/g1000/trace -o trace --output-format csv -- $B --workload groupby --groups 1000 --steps 5 --warmup 1"
    ;;
  *) echo "unknown session $1"; exit 2 ;;
esac
