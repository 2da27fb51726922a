#!/bin/bash
# Round 6: the planner's user passes with the next user's loads in flight -- parity, C3 / C5 lines, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/tl
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_sparse.py tests/test_gpu_exactness.py tests/test_multiproc_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-permuted > $O/c3.json 2> $O/c3.err || { echo "c3 failed"; tail -5 $O/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3 step %.2f span %.2f' % (d['ms_per_step'], d['roofline']['kernel_ms']))"
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { echo "c5 failed"; tail -5 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print('c5 step %.2f count span %.2f topk %.2f' % (d['ms_per_step'], d['roofline']['kernel_ms'], d['topk_ms']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ptl -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find /tmp/ptl -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "tile_" in r["Name"]:
        print("%-40s n=%3s avg=%8.3f ms" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
echo done
