#!/bin/bash
# Round-5 end-of-round GPU steps, selected by PART (each part fits one gpurun call):
#   PART=tests  the whole GPU suite and smoke()
#   PART=bench  the bench lines (C3 with the CPU baseline, C3 with permuted ids, C5, C2) and kernel-trace
#               stats of C3, C5 and C2
#   PART=pmc    PMC passes of k_sp_main (C3), k_rescore (C5) and k_acc_batch (C2)
# Every GPU step has its own time limit; a crash, abort or timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
case "${PART:-tests}" in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; exit $rc
  ;;
bench)
  timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
  timeout -k 10 600 python bench.py --permute-items --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_perm.json 2> gpurun_out/bench_perm.err || exit 1
  timeout -k 10 600 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit 1
  timeout -k 10 600 python bench.py --config c2 --steps 10 --warmup 2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 1
  for f in bench bench_perm bench_c5 bench_c2; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('topk_ms'))"; done
  export TMPDIR=/tmp
  cd /tmp
  for c in c3 c5 c2; do
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_$c" -o run --output-format csv \
      -- python3 "$ROOT/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_$c.log" 2>&1 || exit 1
    echo "rocprof $c ok"
  done
  ;;
pmc)
  SHARDS=8 bash scripts/pmc_sparse.sh || exit 1
  bash scripts/pmc_rescore.sh || exit 1
  bash scripts/pmc_c2.sh || exit 1
  ;;
esac
echo done
