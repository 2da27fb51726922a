set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/bench_c3.py --shards 8 --steps 1 --lib flink-cooccurrence_amd/csrc/libcooc_hip_stats.so > gpurun_out/c3_stats.log 2>&1 || { tail -3 gpurun_out/c3_stats.log; exit 1; }
grep "sp stats" gpurun_out/c3_stats.log | tail -4 | head -2
timeout -k 10 300 python scripts/bench_c3.py --shards 8 --steps 3 > gpurun_out/c3_rel.log 2>&1 || { tail -3 gpurun_out/c3_rel.log; exit 1; }
tail -1 gpurun_out/c3_rel.log | cut -c180-420
