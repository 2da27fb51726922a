set -u
timeout -k 10 600 python -u scripts/bench_stream.py --c3-shard 640 --windows 100 --topk 10 > gpurun_out/stream_c3.json 2> gpurun_out/stream_c3.err || { tail -5 gpurun_out/stream_c3.err; exit 1; }
cat gpurun_out/stream_c3.json
