set -o pipefail
mkdir -p gpurun_out
for v in new head new head; do
  if [ $v = head ]; then export COOC_LIB=flink-cooccurrence_amd/csrc/libcooc_hip_head.so; else unset COOC_LIB; fi
  timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-permuted > gpurun_out/c5_$v.json 2> gpurun_out/c5_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/c5_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c5_$v.json'));r=d.get('roofline_rescore',{});print('$v', 'ms', d['ms_per_step'], 'rescore', {k:r.get(k) for k in ('kernel_ms','achieved','frac')})"
done
unset COOC_LIB
timeout -k 10 900 python -u -m pytest tests/test_gpu_exactness.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_owned_operator_replay.py -m gpu -x -q --timeout 600 > gpurun_out/c5_tests.log 2>&1; rc=$?; tail -3 gpurun_out/c5_tests.log; exit $rc
