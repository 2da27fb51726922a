#!/bin/bash
# A/B of a library variant (flink-cooccurrence_amd/csrc/libcooc_hip_$V.so) against the release build on the
# C3 1/8 shard (scripts/bench_c3.py), after the variant's parity tests (large-universe path).  Each GPU step
# has its own time limit; a crash or timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${V:?variant}
K=${AB_TESTS:-"sparse or exactness"}
if [ "$K" != "none" ]; then
COOC_LIB=flink-cooccurrence_amd/csrc/libcooc_hip_$V.so timeout -k 10 900 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_exactness.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/ab_pytest_$V.log 2>&1
rc=$?; echo "variant $V tests rc=$rc"; tail -3 gpurun_out/ab_pytest_$V.log; [ $rc -eq 0 ] || exit $rc
fi
for lib in release $V release $V; do
  L=flink-cooccurrence_amd/csrc/libcooc_hip_$lib.so; [ $lib = release ] && L=flink-cooccurrence_amd/csrc/libcooc_hip.so
  timeout -k 10 300 python -u scripts/bench_c3.py --steps ${STEPS:-3} --lib $L > gpurun_out/ab_$lib.json 2> gpurun_out/ab_$lib.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $lib rc=$rc"; tail -3 gpurun_out/ab_$lib.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$lib.json'));print('$lib', 'ms', round(d['ms'],2), 'k_sp_main', round(d['k_sp_main_ms'],2), 'pairs/s %.3g' % d['pairs_per_s'])"
done
