set -u
for L in stats t1024; do
timeout -k 10 300 python scripts/bench_c3.py --shards 8 --steps 2 --lib flink-cooccurrence_amd/csrc/libcooc_hip_$L.so > gpurun_out/c3_$L.log 2>&1 || { tail -3 gpurun_out/c3_$L.log; exit 1; }
echo "== $L"; grep "sp stats" gpurun_out/c3_$L.log | tail -3; tail -1 gpurun_out/c3_$L.log | cut -c1-400
done
