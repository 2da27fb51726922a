#!/bin/bash
# GPU tests, then C3 1/8-shard A/B (release vs libcooc_hip_prev.so) and the N = 8 owner simulation of
# one rank with a kernel trace.  Each GPU step has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
TESTS=${TESTS:-all} bash scripts/gpu_r3.sh || exit 1
LIBS="release prev" bash scripts/gpu_abn.sh || exit 1
for lib in release prev; do
  L=$ROOT/flink-cooccurrence_amd/csrc/libcooc_hip_$lib.so; [ $lib = release ] && L=$ROOT/flink-cooccurrence_amd/csrc/libcooc_hip.so
  COOC_LIB=$L timeout -k 10 400 python3 scripts/bench_owner_c3.py --parts 1 --steps 2 > gpurun_out/owner_$lib.json 2> gpurun_out/owner_$lib.err \
    || { echo "owner $lib failed"; tail -3 gpurun_out/owner_$lib.err; exit 1; }
  echo "owner $lib: $(cut -c1-400 gpurun_out/owner_$lib.json)"
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_owner" -o run --output-format csv \
  -- python3 "$ROOT/scripts/bench_owner_c3.py" --parts 1 --steps 2 > "$ROOT/gpurun_out/prof_owner.log" 2>&1 || { echo "rocprof failed"; exit 1; }
echo done
