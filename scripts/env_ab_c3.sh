#!/bin/bash
# Parity of the large-universe path, then the C3 share's time with rank-ordered and permuted ids under two
# settings (VALS, default "0 1") of one environment variable (ABVAR).
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export COOC_BENCH_ANY_ORDER=1
V=${ABVAR:?set ABVAR to the variable to A/B}
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py \
    "tests/test_gpu_exactness.py::test_c3_256th_every_row_vs_record_by_record_oracle" \
    "tests/test_gpu_exactness.py::test_c3_share_every_row_vs_closed_form_oracle" > gpurun_out/rl_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/rl_tests.log; exit 1; }
  tail -2 gpurun_out/rl_tests.log
fi
for rep in 1 2; do
  for v in ${VALS:-0 1}; do
    for p in "" --permute; do
      env $V=$v timeout -k 10 300 python scripts/bench_c3.py --steps 5 $p > gpurun_out/rl_${v}_${rep}${p}.json 2> gpurun_out/rl.err \
        || { echo "bench failed $v $p"; tail -5 gpurun_out/rl.err; exit 1; }
      python3 -c "
import json; d=json.load(open('gpurun_out/rl_${v}_${rep}${p}.json'))
print('$V=$v', 'perm' if d['permuted_ids'] else 'rank', '%.2f ms'%d['ms'], 'k_sp_main %.2f'%d['k_sp_main_ms'], d['check_observed_eq_P'], d['check_sum_rowsum_eq_P'])"
    done
  done
done
