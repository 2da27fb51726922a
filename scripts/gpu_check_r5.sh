# The bounds-checked build (COOC_SP_CHECK) over the benchmark's share (rank-ordered and permuted ids) and
# the sparse suite, then the full-size C2 every-row test on the release build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CHECK=1 bash scripts/gpu_r5.sh || exit $?
CHECK=1 CHECK_ARGS=--permute bash scripts/gpu_r5.sh || exit $?
COOC_LIB=flink-cooccurrence_amd/csrc/libcooc_hip_check.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/check_sparse.log 2>&1
rc=$?; echo "checked sparse suite rc=$rc"; tail -2 gpurun_out/check_sparse.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 600 --timeout-method thread -k c2_every_row > gpurun_out/c2_every_row.log 2>&1
rc=$?; echo "c2 every row rc=$rc"; tail -2 gpurun_out/c2_every_row.log; exit $rc
