# Round-3 bench lines + kernel traces at HEAD for the workloads not re-measured elsewhere
# (filter, G = 1000 group-by, expression scan, Q12 expression / join, hash join).
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1 NUT_COMMIT=$(cat .commit 2>/dev/null)
for w in "filter filter" "groupby1000 groupby --groups 1000" "scanexpr scanexpr" "q12expr q12expr" \
         "q12join q12join" "join join"; do
  set -- $w
  name=$1; shift
  bash scripts/round_measure.sh r03 $name trace --workload "$@" || exit $?
done
