#!/bin/bash
# Planner prefix sums with the u32 list-length table: C3 kernel stats, the bench line, then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/scan3
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/scan3/prof_c3" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config c3 --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/scan3/prof_c3.log" 2>&1) || exit 1
echo "prof ok"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/scan3/bench.json 2> gpurun_out/scan3/bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/scan3/bench.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('permuted', {}).get('ms_per_step'))"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/scan3/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/scan3/pytest_gpu.log; exit $rc
