#!/bin/bash
# Kernel-trace stats of the N=8 owner simulation (rank 0's counting step over the whole log).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/owner_prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
COOC_BENCH_ANY_ORDER=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/po -o run --output-format csv -- python3 $R/scripts/bench_owner_c3.py --world 8 --parts 0 --steps 2 > $R/$O/owner.log 2>&1 || { echo "prof failed"; tail -5 $R/$O/owner.log; exit 1; }
f=$(find /tmp/po -name '*kernel_stats.csv' | head -1)
cp $f $R/$O/kernel_stats_owner.csv
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:24]:
    print("%5s %9.3f ms total  %s" % (r["Calls"], float(r["TotalDurationNs"]) / 1e6, r["Name"][:100]))
PY
echo done
