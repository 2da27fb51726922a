set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python scripts/bench_owner_c3.py --world 8 --parts 0 --steps 1 > gpurun_out/owner_c3.json 2> gpurun_out/owner_c3.err || { tail -5 gpurun_out/owner_c3.err; exit 1; }
cat gpurun_out/owner_c3.json
