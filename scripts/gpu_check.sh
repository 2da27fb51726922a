#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel-trace stats.  Each GPU step has its own
# time limit; a crash / timeout / abort stops the script (no further GPU step in the call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
stop_if_fatal() { # $1 = exit code of a GPU step; test failures (1) are not fatal
  case "$1" in 0|1) ;; *) echo "fatal rc=$1, stopping"; exit "$1";; esac
}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; stop_if_fatal $rc
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$ROOT/gpurun_out/prof.log"; [ $rc -eq 0 ] || exit $rc
fi
echo done
