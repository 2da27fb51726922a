set -u
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -3 gpurun_out/t.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -5 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail -5 gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json
mkdir -p gpurun_out/prof && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o c3 -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || { tail -5 gpurun_out/prof_c3.log; exit 1; }
echo prof done
