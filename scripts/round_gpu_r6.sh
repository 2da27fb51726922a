#!/bin/bash
# Round-6 end-of-round GPU steps, selected by PART (each part fits one gpurun call):
#   PART=tests  the whole GPU suite and smoke()
#   PART=bench  the bench lines (C3 with the CPU baseline and its permuted sub-record, C3 with permuted ids alone,
#               C5 owner unit, C2, C4) and kernel-trace stats of C3, C5 and C2
#   PART=pmc    PMC passes of the C3 counting span, the C5 rescoring passes and k_acc_batch (C2), summarised into
#               gpurun_out/pmc_*.json at these sources' digest
# Every GPU step has its own time limit; a crash, abort or timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
O=$ROOT/gpurun_out/r6
mkdir -p $O
case "${PART:-tests}" in
tests)
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; exit $rc
  ;;
bench)
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
  timeout -k 10 600 python bench.py --permute-items --no-cpu-baseline > $O/bench_perm.json 2> $O/bench_perm.err || exit 1
  timeout -k 10 600 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
  timeout -k 10 600 python bench.py --config c2 --steps 10 --warmup 2 > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
  timeout -k 10 600 python bench.py --config c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
  for f in bench bench_perm bench_c5 bench_c2 bench_c4; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'), d['roofline']['frac'], d.get('topk_ms'), (d.get('permuted') or {}).get('vs_rank_ordered'))"; done
  export TMPDIR=/tmp
  cd /tmp
  for c in c3 c5 c2; do
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$c -o run --output-format csv \
      -- python3 "$ROOT/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-permuted > "$O/prof_$c.log" 2>&1 || exit 1
    cp "$(find /tmp/prof_$c -name '*kernel_stats.csv' | head -1)" "$O/kernel_stats_$c.csv"
    echo "rocprof $c ok"
  done
  ;;
pmc)
  SHARDS=8 bash scripts/pmc_sparse.sh || exit 1
  python3 scripts/pmc_summary.py gpurun_out/pmc_sp $O/pmc_k_sp_main.json 2 > /dev/null || exit 1
  KREGEX='k_rs_score|k_rs_heap' PMC_TAG=pmc_rs PMC_STEPS=1 bash scripts/gpu_r6_pmc_k.sh > /dev/null || exit 1
  cp gpurun_out/pmc_rs/summary.json $O/pmc_k_rescore.json
  bash scripts/pmc_c2.sh || exit 1
  python3 scripts/pmc_summary.py gpurun_out/pmc_c2 $O/pmc_k_acc_batch.json 2 > /dev/null || exit 1
  rm -rf gpurun_out/pmc_sp gpurun_out/pmc_c2
  ls $O
  ;;
esac
echo done
