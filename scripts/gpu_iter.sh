set -u
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -3 gpurun_out/t.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -5 gpurun_out/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c3.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['cpu_baseline']['value'])"
