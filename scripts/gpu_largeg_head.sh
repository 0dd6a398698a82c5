# large-G group-by bench lines at HEAD (full-size parity vs the indexed oracle) + traces
cd $GRAFT_REPO_ROOT && export NUT_PREBUILT=1 NUT_COMMIT=$(cat .commit 2>/dev/null)
bash scripts/round_measure.sh r03 groupby_g1e5 trace --workload groupby --groups 100000 || exit $?
bash scripts/round_measure.sh r03 groupby_g1e7 trace --workload groupby --groups 10000000 || exit $?
