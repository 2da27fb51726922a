#!/bin/bash
# Round 6: k_rs_score timing experiments (results invalid): COOC_RS_EXP=1 no slow entries, 2 no fast-path log, 3 both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/tp4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for e in ${EXPS:-0 1 2 3}; do
  COOC_RS_EXP=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pe$e -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/prof$e.log 2>&1 || { echo "prof failed"; tail -5 $R/$O/prof$e.log; exit 1; }
  f=$(find /tmp/pe$e -name '*kernel_stats.csv' | head -1)
  python3 - "$f" $e <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if "k_rs_" in r["Name"] or "k_rescore" in r["Name"]:
        print("exp %s %-40s n=%5s avg=%10.3f ms" % (sys.argv[2], r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
done
echo done
