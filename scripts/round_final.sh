#!/bin/bash
# Closing evidence of a round at HEAD: Q1 kernel trace + FETCH/WRITE PMC passes + bench
# line, and kernel trace + bench line (CPU baseline, parity, copy floor) for every other
# workload, under gpurun_out/<round>/<name>/ (copy what is judged into profiles/<round>/).
#   scripts/round_final.sh <round>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export NUT_PREBUILT=1 NUT_COMMIT=$(cat .commit 2>/dev/null)
r=${1:?round tag}
bash scripts/round_measure.sh $r q1 pmc --workload q1 || exit $?
for w in "filter filter" "groupby1000 groupby --groups 1000" "groupby1e5 groupby --groups 100000" \
         "groupby1e7 groupby --groups 10000000" "scanexpr scanexpr" "q12expr q12expr" \
         "q12join q12join" "sort sort" "join join"; do
  set -- $w
  name=$1; shift
  bash scripts/round_measure.sh $r $name trace --workload "$@" || exit $?
done
