#!/bin/bash
# Round-5 GPU session (one box): selected steps by env, each GPU step under its own time limit; a crash,
# abort or timeout stops the script (no further GPU step in the call).
#   TESTS=<pytest -k expr | all | none>  TFILES=<test files>  BENCH=1 BENCH_ARGS=...  STATS=1  PROF=1  PMC=1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
fatal() { case "$1" in 0|1) ;; *) echo "fatal rc=$1, stopping"; exit "$1";; esac; }
if [ "${AB:-0}" = "1" ]; then
  # same-box A/B of bench_c3 (rank-ordered and permuted ids): the default build against the env settings in
  # ABENV (";"-separated, e.g. ABENV="COOC_SP_MID=0") and the libraries in ABLIB (space-separated .so paths)
  IFS=';' read -ra ENVS <<< "${ABENV:-}"
  for pass in 1 2; do
    for p in "" ${AB_PERM---permute}; do
      n=rank; [ -n "$p" ] && n=perm
      i=0
      for e in "" "${ENVS[@]}"; do
        env $e timeout -k 10 300 python -u scripts/bench_c3.py --steps 3 $p > gpurun_out/ab_${n}_$i.json 2> gpurun_out/ab_${n}_$i.err || { echo "ab failed: $e"; tail -3 gpurun_out/ab_${n}_$i.err; exit 1; }
        python -c "import json;d=json.load(open('gpurun_out/ab_${n}_$i.json'));print('$n [$e]', 'ms', round(d['ms'],2), 'span', round(d['k_sp_main_ms'],2), 'nnz', d['nnz'], d['verify']['rows_bad_sum'], d['verify']['rows_bad_entries'])"
        i=$((i+1))
      done
      for l in ${ABLIB:-}; do
        timeout -k 10 300 python -u scripts/bench_c3.py --steps 3 $p --lib $l > gpurun_out/ab_${n}_lib.json 2> gpurun_out/ab_${n}_lib.err || { echo "ab failed: $l"; exit 1; }
        python -c "import json;d=json.load(open('gpurun_out/ab_${n}_lib.json'));print('$n [$l]', 'ms', round(d['ms'],2), 'span', round(d['k_sp_main_ms'],2), 'nnz', d['nnz'], d['verify']['rows_bad_sum'], d['verify']['rows_bad_entries'])"
      done
    done
  done
fi
if [ "${SORTB:-0}" = "1" ]; then
  for v in 0 ${SORTB_HIPCUB:-}; do
    COOC_SR_HIPCUB=$v timeout -k 10 600 python -u scripts/bench_c3.py --steps 2 --planner sort > gpurun_out/sort_$v.json 2> gpurun_out/sort_$v.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/sort_$v.json'));print('sort hipcub=$v ms', round(d['ms'],1), 'rows,pairs', d['sort_path_rows_pairs'], 'verify', d['verify']['rows_bad_sum'], d['verify']['rows_bad_entries'], d['nnz'])"
  done
fi
T=${TESTS:-none}
if [ "$T" != "none" ]; then
  K=(); [ "$T" != "all" ] && K=(-k "$T")
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TFILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|FAIL" gpurun_out/pytest_gpu.log | tail -8; fatal $rc
  [ $rc -eq 0 ] || exit 1
fi
if [ "${SMOKE:-0}" = "1" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 600 python -u bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.err
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'k_ms',r['kernel_ms'],'frac',r['frac'],'cpu',(d.get('cpu_baseline') or {}).get('value'))"
fi
if [ "${STATS:-0}" = "1" ]; then
  for p in "" ${STATS_PERM:-}; do
  timeout -k 10 300 python -u scripts/bench_c3.py --steps 2 $p --lib flink-cooccurrence_amd/csrc/libcooc_hip_stats.so \
    > gpurun_out/phase_stats$p.txt 2>&1
  rc=$?; echo "stats $p rc=$rc"; grep "sp stats" gpurun_out/phase_stats$p.txt | tail -8; [ $rc -eq 0 ] || exit $rc
  done
fi
if [ "${CHECK:-0}" = "1" ]; then
  # the bounds-checked build (COOC_SP_CHECK: every guarded global index sets err bit 8 instead of faulting)
  timeout -k 10 300 python -u scripts/bench_c3.py --steps 2 ${CHECK_ARGS:-} --lib flink-cooccurrence_amd/csrc/libcooc_hip_check.so \
    > gpurun_out/check.json 2> gpurun_out/check.err
  rc=$?; echo "check rc=$rc"; tail -2 gpurun_out/check.err; cat gpurun_out/check.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROF:-0}" = "1" ]; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$ROOT/gpurun_out/prof.log" 2>&1)
  rc=$?; echo "rocprof rc=$rc"; tail -1 "$ROOT/gpurun_out/prof.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
fi
if [ "${KPROF:-0}" = "1" ]; then
  # per-kernel times of one C3 share count (scripts/bench_c3.py) under rocprofv3 --kernel-trace --stats
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/kprof" -o run --output-format csv \
    -- python3 "$ROOT/scripts/bench_c3.py" --steps 2 ${KPROF_ARGS:-} > "$ROOT/gpurun_out/kprof.log" 2>&1)
  rc=$?; echo "kprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - "$ROOT/gpurun_out/kprof" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e6:8.3f} ms')
PY
fi
if [ "${PMCIC:-0}" = "1" ]; then
  bash scripts/pmc_icache.sh || exit 1
fi
if [ "${PMC:-0}" = "1" ]; then
  bash scripts/pmc_sparse.sh || exit 1
  python3 scripts/pmc_summary.py gpurun_out/pmc_sp gpurun_out/pmc_k_sp_main.json
fi
echo done
