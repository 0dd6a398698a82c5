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
  s3)  # G = 1000: the shared table's slots per group x workgroups per CU
    G="$B --workload groupby --groups 1000"
    scripts/gpu_session.sh \
      "200 g_def $G" "200 g_s2 $G --option agg_slots=2" "200 g_s2b3 $G --option agg_slots=2 --option agg_blocks=3" \
      "200 g_s8 $G --option agg_slots=8" "200 g_def2 $G" "200 g_s2b $G --option agg_slots=2" \
      "200 g_s2b2 $G --option agg_slots=2 --option agg_blocks=2"
    ;;
  s4)  # G = 1000 after the one-wait tail: plain runs, SQ / LDS counters of the agg kernel
    mkdir -p gpurun_out/g1000
    G="$B --workload groupby --groups 1000"
    scripts/gpu_session.sh \
      "200 g4_a $G" "200 g4_b $G" \
      "120 g4_sq timeout -s KILL 110 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d gpurun_out/g1000/sq -o sq --output-format csv -- $G --steps 3 --warmup 1" \
      "120 g4_sq2 timeout -s KILL 110 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY -d gpurun_out/g1000/sq2 -o sq --output-format csv -- $G --steps 3 --warmup 1" \
      "200 q1_a $B --workload q1"
    ;;
  s5)  # G = 1000: bucket vs own-slot LDS lookups, interleaved
    G="$B --workload groupby --groups 1000"
    scripts/gpu_session.sh \
      "200 h0a $G" "200 h1a $G --option agg_home=1" "200 h0b $G" "200 h1b $G --option agg_home=1" \
      "200 h1s8 $G --option agg_home=1 --option agg_slots=8" "200 h1s2 $G --option agg_home=1 --option agg_slots=2" \
      "200 g1e5h1 $B --workload groupby --groups 100000 --option agg_home=1" "200 g1e5h0 $B --workload groupby --groups 100000"
    ;;
  s6)  # G = 1e7 ordered: CUs the level-1 scatter leaves to the aggregation
    G="$B --workload groupby --groups 10000000"
    scripts/gpu_session.sh \
      "200 e0a $G" "200 e16 $G --option gb_l1_spare=16" "200 e32 $G --option gb_l1_spare=32" \
      "200 e64 $G --option gb_l1_spare=64" "200 e0b $G" "200 e32b $G --option gb_l1_spare=32" \
      "200 e48 $G --option gb_l1_spare=48"
    ;;
  s7)  # G = 1e7 ordered: one step's timeline (kernels + copies)
    mkdir -p gpurun_out/g1e7
    scripts/gpu_session.sh \
      "300 e_trace rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/g1e7/trace -o trace --output-format csv -- $B --workload groupby --groups 10000000 --steps 3 --warmup 1 --no-copy-floor --option gb_l1_spare=32"
    ;;
  s8)  # G = 1e7 / Zipf with the ordering on its own stream; gorder tests first
    G="$B --workload groupby --groups 10000000"
    scripts/gpu_session.sh \
      "400 t_gorder $T tests/test_gpu_gorder.py" \
      "200 f0 $G" "200 f32 $G --option gb_l1_spare=32" "200 f0b $G" "200 f32b $G --option gb_l1_spare=32" \
      "200 fz32 $G --skew --option gb_l1_spare=32" "200 fz0 $G --skew" \
      "200 f1e5 $B --workload groupby --groups 100000"
    ;;
  s9)  # the library's multi-GPU path at one RCCL rank (bench --dist) next to the plain lines
    scripts/gpu_session.sh \
      "200 d_q1 $B --workload q1 --dist" "200 p_q1 $B --workload q1" \
      "200 d_g1000 $B --workload groupby --groups 1000 --dist" \
      "200 d_g1e5 $B --workload groupby --groups 100000 --dist" \
      "200 d_filter $B --workload filter --dist" "300 d_sort $B --workload sort --dist" \
      "300 d_join $B --workload join --dist"
    ;;
  s10)  # dist tests after the P = 1 join / filter shortcuts, and their --dist lines
    scripts/gpu_session.sh \
      "500 t_dist $T tests/test_gpu_dist_native.py tests/test_gpu_join.py" \
      "200 d_filter2 $B --workload filter --dist" "300 d_join2 $B --workload join --dist"
    ;;
  *) echo "unknown session $1"; exit 2 ;;
esac
