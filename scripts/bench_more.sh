#!/bin/bash
# C4 streaming and C5-at-C2-scale measurements (one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python scripts/bench_topk.py --topk 50 > gpurun_out/bench_topk.json 2> gpurun_out/bench_topk.err
rc=$?; echo "topk rc=$rc"; cat gpurun_out/bench_topk.json; tail -3 gpurun_out/bench_topk.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_stream.py --windows 100 > gpurun_out/bench_stream.json 2> gpurun_out/bench_stream.err
rc=$?; echo "stream rc=$rc"; cat gpurun_out/bench_stream.json; tail -3 gpurun_out/bench_stream.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_stream.py --windows 100 --topk 50 --copy > gpurun_out/bench_stream_topk.json 2> gpurun_out/bench_stream_topk.err
rc=$?; echo "stream+topk rc=$rc"; cat gpurun_out/bench_stream_topk.json; tail -3 gpurun_out/bench_stream_topk.err; [ $rc -eq 0 ] || exit $rc
