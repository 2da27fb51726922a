#!/bin/bash
# Round 6: the two-pass rescoring (k_rs_bounds / k_rs_score / k_rs_heap) -- parity with whole-log row sums (its
# default) and forced on every CSR rescoring test (COOC_RS_TWO_PASS=1), then C5 owner-unit timing against
# k_rescore3 (COOC_RS_TWO_PASS=0) and a kernel-trace profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tp
mkdir -p $O
T="tests/test_gpu_sparse.py::test_c5_topk_c3_shape_vs_oracle tests/test_gpu_sparse.py::test_c5_topk_long_rows_vs_oracle \
  tests/test_gpu_sparse.py::test_c5_topk_owned_parts_vs_whole tests/test_gpu_parity.py::test_batch_topk_vs_rescorer \
  tests/test_gpu_parity.py::test_c2_scale_topk_rows"
COOC_RS_TWO_PASS=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $T > $O/tests_forced.log 2>&1 || { echo "forced tests failed"; tail -40 $O/tests_forced.log; exit 1; }
echo "forced tests ok"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_exactness.py::test_c5_owner_unit_vs_oracle > $O/tests_owner.log 2>&1 || { echo "owner test failed"; tail -40 $O/tests_owner.log; exit 1; }
echo "owner test ok"
for rep in 1 2; do
  for v in 0 1; do
    COOC_RS_TWO_PASS=$v timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_tp${v}_$rep.json 2> $O/c5.err || { echo "c5 bench failed $v"; tail -5 $O/c5.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c5_tp${v}_$rep.json')); print('c5 tp$v', 'step %.2f'%d['ms_per_step'], 'topk %.2f'%d['topk_ms'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof failed"; tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/$O/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print("%-60s n=%5s avg=%10.3f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
echo done
