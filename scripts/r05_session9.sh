#!/bin/bash
# Round 5 session 9: Zipf mismatch localisation; chain computed-key gather fix (fixture 9).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "200 skewdbg python -u scripts/diag/skew_debug.py" \
  "300 t_sub python -u -m pytest tests/test_gpu_substring.py tests/test_gpu_subquery.py -q --timeout 200 --timeout-method thread" \
  "400 t_gorder python -u -m pytest tests/test_gpu_gorder.py -q --timeout 200 --timeout-method thread"
