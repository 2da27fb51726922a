#!/bin/bash
# A/B of accumulate variants on one box: parity tests on the default variant, then one bench per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  case $rc in 0|1) ;; *) exit $rc;; esac
fi
for v in ${VARIANTS:-1 2}; do
  COOC_ACC_VARIANT=$v timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err
  rc=$?; echo "variant $v rc=$rc"; python3 -c "
import json,sys; d=json.load(open('gpurun_out/bench_v$v.json')); r=d['roofline']
print('v$v', '%.3e pairs/s'%d['value'], '%.2f ms/step'%d['ms_per_step'], 'kernel %.2f ms'%r['kernel_ms'], 'frac %.3f'%r['frac'])" || tail -5 gpurun_out/bench_v$v.err
  [ $rc -eq 0 ] || exit $rc
done
