#!/bin/bash
# Round 5 session 22: exact key scatter cost vs bin count (the sort-fold question, §6).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh "200 bins_tune scripts/tune/bin/bins_tune"
