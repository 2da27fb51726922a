#!/bin/bash
# C5 rescoring time (bench.py --config c5 topk_ms) over library variants built by scripts/build_variant.sh:
# LIBS="rsA rsB ..." (release = the in-tree build), two rounds.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in release ${LIBS}; do
    L=""; [ "$v" != release ] && L=$(pwd)/flink-cooccurrence_amd/csrc/libcooc_hip_$v.so
    COOC_LIB=$L timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/rsab_${v}_$rep.json 2> gpurun_out/rsab.err || { echo "bench failed $v"; tail -5 gpurun_out/rsab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/rsab_${v}_$rep.json')); print('$v', 'topk_ms %.2f'%d['topk_ms'], 'step %.2f'%d['ms_per_step'])"
  done
done
