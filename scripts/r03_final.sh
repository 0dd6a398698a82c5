# Round-3 closing evidence at HEAD: Q1 kernel trace + FETCH/WRITE PMC passes + bench line,
# and kernel trace + bench line (CPU baseline, parity, copy floor) for every other workload
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1 NUT_COMMIT=$(cat .commit 2>/dev/null)
bash scripts/round_measure.sh r03 q1 pmc --workload q1 || exit $?
for w in "filter filter" "groupby1000 groupby --groups 1000" "scanexpr scanexpr" "q12expr q12expr" \
         "q12join q12join" "sort sort" "join join"; do
  set -- $w
  name=$1; shift
  bash scripts/round_measure.sh r03 $name trace --workload "$@" || exit $?
done
