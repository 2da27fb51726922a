#!/bin/bash
# The whole GPU suite (as the driver runs it) plus smoke(), at the working tree's build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/suite
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -2 $O/smoke.log
exit $rc
