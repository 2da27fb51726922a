set -u
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
timeout -k 10 600 python scripts/bench_owner_c3.py --world 8 --parts 0 --steps 2 > gpurun_out/owner_c3.json 2> gpurun_out/owner_c3.err || { tail -5 gpurun_out/owner_c3.err; exit 1; }
cat gpurun_out/owner_c3.json
