set -u
timeout -k 10 300 python scripts/bench_c3.py --shards 8 --steps 1 --lib flink-cooccurrence_amd/csrc/libcooc_hip_stats.so > gpurun_out/c3_stats.log 2>&1 || { tail -3 gpurun_out/c3_stats.log; exit 1; }
grep "sp stats" gpurun_out/c3_stats.log | tail -4
