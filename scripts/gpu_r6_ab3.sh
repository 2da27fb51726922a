#!/bin/bash
# Round 6 A/B 3: k_rescore3 with the heap in registers (COOC_RS_V=4) vs in LDS (3); timing experiments (results
# invalid): COOC_RS_EXP=1 no heap, 2 no scoring.  Rescoring tests with V=4 first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab3
mkdir -p $O
COOC_RS_V=4 timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_exactness.py::test_c5_owner_unit_vs_oracle \
  tests/test_gpu_sparse.py::test_c5_topk_c3_shape_vs_oracle tests/test_gpu_sparse.py::test_c5_topk_long_rows_vs_oracle \
  tests/test_gpu_sparse.py::test_c5_topk_owned_parts_vs_whole tests/test_gpu_sparse.py::test_streaming_sparse_global_rows_vs_oracle \
  tests/test_gpu_parity.py::test_batch_topk_vs_rescorer tests/test_gpu_parity.py::test_c2_scale_topk_rows > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
echo "tests ok"
for rep in 1 2; do
  for v in v3 v4 v4e1 v4e2 v3e1; do
    case $v in v3) env="COOC_RS_V=3";; v4) env="COOC_RS_V=4";; v4e1) env="COOC_RS_V=4 COOC_RS_EXP=1";; v4e2) env="COOC_RS_V=4 COOC_RS_EXP=2";; v3e1) env="COOC_RS_V=3 COOC_RS_EXP=1";; esac
    env $env timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5.err || { echo "c5 bench failed $v"; tail -5 $O/c5.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); print('c5 $v', 'step %.2f'%d['ms_per_step'], 'topk %.2f'%d['topk_ms'])"
  done
done
echo done
