#!/bin/bash
# Round 6: k_rs_score variants (COOC_LIB builds from scripts/build_variant.sh) on the C5 owner unit, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/tp5
mkdir -p $O
COOC_RS_TWO_PASS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py::test_c5_topk_long_rows_vs_oracle tests/test_gpu_parity.py::test_batch_topk_vs_rescorer > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests ok"
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-release}; do
  lib=$R/flink-cooccurrence_amd/csrc/libcooc_hip.so
  [ "$v" != release ] && lib=$R/flink-cooccurrence_amd/csrc/libcooc_hip_$v.so
  COOC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pv$v -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/prof_$v.log 2>&1 || { echo "prof failed"; tail -5 $R/$O/prof_$v.log; exit 1; }
  f=$(find /tmp/pv$v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rs_" in r["Name"] or "k_rescore" in r["Name"]:
        print("%s %-40s n=%5s avg=%10.3f ms" % (sys.argv[2], r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
done
echo done
