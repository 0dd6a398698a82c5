#!/bin/bash
# round_final.sh split over several gpurun calls (each within the call limit):
#   scripts/round_final_part.sh <round> <part 1|2|3>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export NUT_PREBUILT=1 NUT_COMMIT=$(cat .commit 2>/dev/null)
r=${1:?round tag}
case "$2" in
  1) bash scripts/round_measure.sh $r q1 pmc --workload q1 || exit $?
     set -- "filter filter" "groupby1000 groupby --groups 1000" ;;
  2) set -- "groupby1e5 groupby --groups 100000" "groupby1e7 groupby --groups 10000000" \
       "groupby1e7zipf groupby --groups 10000000 --skew" "sort sort" ;;
  3) set -- "scanexpr scanexpr" "q12expr q12expr" "q12join q12join" "join join" ;;
  4) bash scripts/round_measure.sh $r sort_pmc pmc --workload sort || exit $?
     exit 0 ;;
  5) bash scripts/round_measure.sh $r join_pmc pmc --workload join || exit $?
     exit 0 ;;
  *) echo "part 1|2|3|4|5"; exit 2 ;;
esac
for w in "$@"; do
  set -- $w
  name=$1; shift
  bash scripts/round_measure.sh $r $name trace --workload "$@" || exit $?
done
