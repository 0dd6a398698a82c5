#!/bin/bash
# Round 5 session 12: heavy-pass harness (where its 11 ms go).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_session.sh \
  "200 hk_tune scripts/tune/bin/hk_tune"
