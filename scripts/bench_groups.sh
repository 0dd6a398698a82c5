#!/bin/bash
# config 3 cardinality sweep: one bench line per G (stderr kept in gpurun_out/bench_groups.err)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for g in "$@"; do
  timeout -k 10 240 python bench.py --workload groupby --groups "$g" --no-cpu-baseline --steps 5 \
    2>>gpurun_out/bench_groups.err | tail -1 || exit $?
done
