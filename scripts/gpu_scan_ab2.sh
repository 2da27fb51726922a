#!/bin/bash
# Planner prefix sums: blocked (default) vs LDS-staged tiles, C3 kernel stats of each; then the streaming and
# sparse GPU tests at the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/scan2
export TMPDIR=/tmp
for v in 1 0; do
  (cd /tmp && COOC_SCAN_BLOCKED=$v timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/scan2/prof_c3_b$v" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config c3 --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/scan2/prof_c3_b$v.log" 2>&1) || exit 1
  echo "prof b$v ok"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_sparse.py tests/test_streaming_multiproc.py tests/test_gpu_parity.py tests/test_multiproc_gpu.py tests/test_owned_operator_replay.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/scan2/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/scan2/pytest_gpu.log; exit $rc
