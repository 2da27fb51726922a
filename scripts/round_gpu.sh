#!/bin/bash
# Full GPU session: tests, unroll A/B, kernel-trace profile, PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/ab_unroll.sh || exit $?
SKIP_TESTS=1 SKIP_BENCH=1 bash scripts/gpu_check.sh || exit $?
bash scripts/pmc.sh || exit $?
