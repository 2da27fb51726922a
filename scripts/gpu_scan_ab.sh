#!/bin/bash
# Hand-written planner prefix sums (cooc_scan.h): the GPU suite, the C3 bench line and its kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/scan
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/scan/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/scan/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/scan/bench.json 2> gpurun_out/scan/bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/scan/bench.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('permuted', {}).get('ms_per_step'))"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/scan/prof_c3" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config c3 --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/scan/prof_c3.log" 2>&1 || exit 1
echo done
