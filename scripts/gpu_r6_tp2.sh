#!/bin/bash
# Round 6: kernel-trace stats of the C5 owner unit with the two-pass rescoring (only the stats kept).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/tp2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${TP_VARIANTS:-1}; do
  COOC_RS_TWO_PASS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof$v -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/prof$v.log 2>&1 || { echo "prof failed"; tail -5 $R/$O/prof$v.log; exit 1; }
  f=$(find /tmp/prof$v -name '*kernel_stats.csv' | head -1)
  cp "$f" $R/$O/kernel_stats_tp$v.csv
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print("%-60s n=%5s avg=%10.3f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
done
echo done
