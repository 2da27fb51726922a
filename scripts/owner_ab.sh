# N = 8 owner simulation, the release build against another library (OWNER_LIB), ranks 1 and 0, twice;
# then the owned-row GPU tests.
set -o pipefail
mkdir -p gpurun_out
export COOC_BENCH_ANY_ORDER=1
for pass in 1 2; do
  for l in "" ${OWNER_LIB:-}; do
    a=(); [ -n "$l" ] && a=(--lib $l)
    timeout -k 10 600 python -u scripts/bench_owner_c3.py --world 8 --parts 1,0 --steps 3 "${a[@]}" > gpurun_out/owner_ab.json 2> gpurun_out/owner_ab.err || { echo "owner sim failed"; tail -3 gpurun_out/owner_ab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/owner_ab.json'));print('[$l]', {p:(round(v['ms'],2), round(v['k_sp_main_ms'],2)) for p,v in d['parts'].items()})"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_sparse.py tests/test_multiproc_gpu.py tests/test_owned_operator_replay.py -m gpu -x -q --timeout 600 -k "owned or multiproc or two or replay" > gpurun_out/owner_tests.log 2>&1
rc=$?; tail -2 gpurun_out/owner_tests.log; exit $rc
