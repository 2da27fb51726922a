#!/bin/bash
# Round 6: k_rs_heap's tail -- timing experiments (results invalid) skipping rows longer than COOC_RS_HEAP_SKIP.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
cd /tmp && export TMPDIR=/tmp
for sk in ${SKIPS:-0 1000000 262144 65536}; do
  COOC_RS_HEAP_SKIP=$sk timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ph$sk -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > /tmp/ph$sk.log 2>&1 || { echo "prof failed"; tail -5 /tmp/ph$sk.log; exit 1; }
  f=$(find /tmp/ph$sk -name '*kernel_stats.csv' | head -1)
  python3 - "$f" $sk <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rs_heap" in r["Name"]:
        print("skip>%s %-20s avg=%8.3f ms" % (sys.argv[2], r["Name"][:20], float(r["AverageNs"]) / 1e6))
PY
done
python3 - <<'PY'
PY
echo done
