#!/bin/bash
# C5 on one GPU (parity tests, bench --config c5, kernel trace), then the k_sp_main PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -x -v --timeout 300 --timeout-method thread -k "c5" \
  > gpurun_out/pytest_c5.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_c5.log; exit 1; }
tail -3 gpurun_out/pytest_c5.log
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err \
  || { echo "bench rc=$?"; tail -5 gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_c5" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_c5.log" 2>&1 \
  || { echo "rocprof rc=$?"; exit 1; }
cd "$ROOT"
if [ -f flink-cooccurrence_amd/csrc/libcooc_hip_stats.so ]; then
  timeout -k 10 300 python scripts/bench_c3.py --shards 8 --steps 1 --lib flink-cooccurrence_amd/csrc/libcooc_hip_stats.so \
    > gpurun_out/c3_stats.log 2>&1 || { echo "stats rc=$?"; exit 1; }
  grep "sp stats" gpurun_out/c3_stats.log | tail -2
fi
if [ "${PMC:-1}" = "1" ]; then bash scripts/pmc_sparse.sh || exit $?; fi
echo done
