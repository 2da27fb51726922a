#!/bin/bash
# Round 6 A/B: wave chunks (k_sp_main, COOC_SP_WAVE) and the pipelined rescoring kernel (k_rescore2, COOC_RS_V2)
# against the previous build (libcooc_hip_old.so).  Correctness of the new build first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab1
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  "tests/test_gpu_exactness.py::test_c3_share_every_row_vs_closed_form_oracle[8-False-True]" \
  "tests/test_gpu_exactness.py::test_c3_share_every_row_vs_closed_form_oracle[64-True-True]" \
  tests/test_gpu_exactness.py::test_c5_owner_unit_vs_oracle > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests ok"
L=$(pwd)/flink-cooccurrence_amd/csrc
for rep in 1 2; do
  for v in old new new_w0; do
    case $v in old) lib=$L/libcooc_hip_old.so; env="";; new) lib=$L/libcooc_hip.so; env="";; new_w0) lib=$L/libcooc_hip.so; env="COOC_SP_WAVE=0";; esac
    env $env COOC_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-permuted > $O/c3_${v}_$rep.json 2> $O/c3.err || { echo "c3 bench failed $v"; tail -5 $O/c3.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c3_${v}_$rep.json')); print('c3 $v', 'step %.2f'%d['ms_per_step'], 'span %.2f'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
for rep in 1 2; do
  for v in old new new_v1; do
    case $v in old) lib=$L/libcooc_hip_old.so; env="";; new) lib=$L/libcooc_hip.so; env="";; new_v1) lib=$L/libcooc_hip.so; env="COOC_RS_V2=0";; esac
    env $env COOC_LIB=$lib timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5.err || { echo "c5 bench failed $v"; tail -5 $O/c5.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); print('c5 $v', 'step %.2f'%d['ms_per_step'], 'span %.2f'%d['roofline']['kernel_ms'], 'topk %.2f'%d['topk_ms'])"
  done
done
echo done
