#!/bin/bash
# Round 6: two-pass rescoring -- parity (forced on the CSR rescoring tests, default on the C5 owner unit), then
# kernel-trace stats of the C5 owner unit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tp3
mkdir -p $O
T="tests/test_gpu_sparse.py::test_c5_topk_c3_shape_vs_oracle tests/test_gpu_sparse.py::test_c5_topk_long_rows_vs_oracle \
  tests/test_gpu_sparse.py::test_c5_topk_owned_parts_vs_whole tests/test_gpu_parity.py::test_batch_topk_vs_rescorer tests/test_gpu_configs.py::test_device_llr_known_answers tests/test_gpu_configs.py::test_device_llr_bit_exact_vs_oracle tests/test_gpu_split_heap.py"
COOC_RS_TWO_PASS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $T > $O/tests_forced.log 2>&1 || { echo "forced tests failed"; tail -40 $O/tests_forced.log; exit 1; }
echo "forced tests ok"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_exactness.py::test_c5_owner_unit_vs_oracle > $O/tests_owner.log 2>&1 || { echo "owner test failed"; tail -40 $O/tests_owner.log; exit 1; }
echo "owner test ok"
TP_VARIANTS="${TP_VARIANTS:-1}" bash scripts/gpu_r6_tp2.sh
