#!/bin/bash
# A/B the bench over environment settings: AB="NAME=v1 NAME=v2,OTHER=w ..." (one bench per setting;
# commas join several variables of one setting)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for kv in ${AB}; do
  i=$((i+1))
  env ${kv//,/ } timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "$kv rc=$rc"; tail -5 gpurun_out/ab_$i.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$i.json')); r=d['roofline']
print('$kv', '%.3e pairs/s'%d['value'], '%.2f ms/step'%d['ms_per_step'], 'kernel %.2f ms'%r['kernel_ms'], 'frac %.3f'%r['frac'])"
done
