#!/bin/bash
# Round 6 A/B 2: the LDS-DMA rescoring kernel (k_rescore3, COOC_RS_V=3) against k_rescore2 / k_rescore and the
# previous build, on the C5 owner unit; the rescoring tests at the new build first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_exactness.py::test_c5_owner_unit_vs_oracle tests/test_gpu_exactness.py::test_c5_topk_benched_share_vs_oracle \
  tests/test_gpu_sparse.py::test_c5_topk_c3_shape_vs_oracle tests/test_gpu_sparse.py::test_c5_topk_long_rows_vs_oracle \
  tests/test_gpu_sparse.py::test_c5_topk_owned_parts_vs_whole tests/test_gpu_sparse.py::test_streaming_sparse_global_rows_vs_oracle \
  tests/test_gpu_parity.py::test_batch_topk_vs_rescorer tests/test_gpu_parity.py::test_c2_scale_topk_rows \
  tests/test_gpu_parity.py::test_streaming_windows_vs_oracle > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
echo "tests ok"
L=$(pwd)/flink-cooccurrence_amd/csrc
for rep in 1 2; do
  for v in old v3 v2 v1; do
    case $v in old) lib=$L/libcooc_hip_old.so; env="COOC_RS_V=1";; v3) lib=$L/libcooc_hip.so; env="COOC_RS_V=3";; v2) lib=$L/libcooc_hip.so; env="COOC_RS_V=2";; v1) lib=$L/libcooc_hip.so; env="COOC_RS_V=1";; esac
    env $env COOC_LIB=$lib timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5.err || { echo "c5 bench failed $v"; tail -5 $O/c5.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); print('c5 $v', 'step %.2f'%d['ms_per_step'], 'span %.2f'%d['roofline']['kernel_ms'], 'topk %.2f'%d['topk_ms'], 'read %.3f'%d['c5_regime']['entries_read_frac'])"
  done
done
COOC_RS_NO_NAN_EXIT=1 timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_v3_full.json 2> $O/c5.err && python3 -c "import json; d=json.load(open('$O/c5_v3_full.json')); print('c5 v3 full scoring', 'topk %.2f'%d['topk_ms'])"
echo done
