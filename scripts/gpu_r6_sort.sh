#!/bin/bash
# Round 6: the planner's hand-written sorts (cooc_radix.h) -- radix tests, the large-universe parity tests, then the
# C3 line with the hand-written sorts (default) and the library ones (COOC_LIB_SORTS=1), and kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/sort
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_radix.py tests/test_gpu_sparse.py tests/test_gpu_exactness.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in 0 1; do
    COOC_LIB_SORTS=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-permuted > $O/c3_lib${v}_$rep.json 2> $O/c3.err || { echo "bench failed"; tail -5 $O/c3.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c3_lib${v}_$rep.json')); print('lib$v', 'step %.2f'%d['ms_per_step'], 'span %.2f'%d['roofline']['kernel_ms'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ps -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-permuted > $R/$O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find /tmp/ps -name '*kernel_stats.csv' | head -1)
cp $f $R/$O/kernel_stats_c3.csv
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "rdx" in n or "select" in n or "rocprim" in n or "scan_lookback" in n:
        print("%-70s n=%4s total=%8.3f ms" % (n[:70], r["Calls"], float(r["TotalDurationNs"]) / 1e6))
PY
echo done
