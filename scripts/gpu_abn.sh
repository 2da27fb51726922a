#!/bin/bash
# Timing A/B of several library builds on the C3 1/8 shard (scripts/bench_c3.py), interleaved twice.
# LIBS="release fix noret ..." (release = libcooc_hip.so, else libcooc_hip_<name>.so).  Each run has its
# own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pass in 1 2; do
  for lib in ${LIBS:?}; do
    L=flink-cooccurrence_amd/csrc/libcooc_hip_$lib.so; [ $lib = release ] && L=flink-cooccurrence_amd/csrc/libcooc_hip.so
    timeout -k 10 300 python -u scripts/bench_c3.py --shards ${SHARDS:-8} --steps ${STEPS:-3} --lib $L > gpurun_out/abn_$lib.json 2> gpurun_out/abn_$lib.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $lib rc=$rc"; tail -3 gpurun_out/abn_$lib.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/abn_$lib.json'));print('$lib', 'ms', round(d['ms'],2), 'k_sp_main', round(d['k_sp_main_ms'],2), 'pairs/s %.3g' % d['pairs_per_s'])"
  done
done
