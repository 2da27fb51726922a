#!/bin/bash
# Round-end GPU session: parity tests, the three bench lines (C3 default, C5, C2), kernel-trace
# stats of C3 and C5, and the k_sp_main PMC passes.  Each GPU step has its own time limit; a crash,
# abort or timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; case $rc in 0|1) ;; *) exit $rc;; esac
fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
timeout -k 10 600 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit 1
timeout -k 10 600 python bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 1
for f in bench bench_c5 bench_c2; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('topk_ms'))"; done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_c3" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_c3.log" 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_c5" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_c5.log" 2>&1 || exit 1
cd "$ROOT"
bash scripts/pmc_sparse.sh || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc_sp gpurun_out/pmc_k_sp_main.json > /dev/null
echo done
