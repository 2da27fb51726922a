#!/bin/bash
# Timing experiment on C5's rescoring kernel (k_rescore): release build vs libcooc_hip_rs1.so (heap only
# filled, never replaced) and libcooc_hip_rs2.so (column-table gathers confined to 1024 columns).  The
# variants' heaps are NOT the reference's; only topk_ms is read.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in release ${VARIANTS:-rs1 rs2}; do
  L=flink-cooccurrence_amd/csrc/libcooc_hip_$lib.so; [ $lib = release ] && L=flink-cooccurrence_amd/csrc/libcooc_hip.so
  COOC_LIB=$L timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rs_$lib.json 2> gpurun_out/rs_$lib.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $lib rc=$rc"; tail -3 gpurun_out/rs_$lib.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/rs_$lib.json'));print('$lib', 'ms', round(d['ms_per_step'],2), 'topk_ms', round(d['topk_ms'],2))"
done
