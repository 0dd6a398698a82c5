#!/bin/bash
# Round 5 session 24: HBM traffic per step (FETCH_SIZE / WRITE_SIZE passes) of the
# partitioned group-by lines: G = 1e5, G = 1e7 uniform and Zipf-like.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export NUT_PREBUILT=1 NUT_COMMIT=$(cat .commit 2>/dev/null)
bash scripts/round_measure.sh r05 g1e5_pmc pmc --workload groupby --groups 100000 || exit $?
bash scripts/round_measure.sh r05 g1e7_pmc pmc --workload groupby --groups 10000000 || exit $?
bash scripts/round_measure.sh r05 g1e7z_pmc pmc --workload groupby --groups 10000000 --skew || exit $?
