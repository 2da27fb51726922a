#!/bin/bash
# Kernel trace of bench.py --config c5 for the release build and the variants in $VARIANTS
# (flink-cooccurrence_amd/csrc/libcooc_hip_<v>.so); per-kernel stats under gpurun_out/rsprof_<v>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in release ${VARIANTS:-}; do
  L=$ROOT/flink-cooccurrence_amd/csrc/libcooc_hip_$lib.so; [ $lib = release ] && L=$ROOT/flink-cooccurrence_amd/csrc/libcooc_hip.so
  cd /tmp
  COOC_LIB=$L timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/rsprof_$lib" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config c5 --steps 2 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/rsprof_$lib.log" 2>&1
  rc=$?; cd "$ROOT"; [ $rc -eq 0 ] || { echo "rocprof $lib rc=$rc"; tail -5 gpurun_out/rsprof_$lib.log; exit $rc; }
  f=$(ls gpurun_out/rsprof_$lib/*/run_kernel_stats.csv gpurun_out/rsprof_$lib/run_kernel_stats.csv 2>/dev/null | head -1)
  echo "== $lib"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:8]: print(r['Name'][:60], r['Calls'], '%.2f ms avg' % (float(r['AverageNs'])/1e6))"
done
