set -u
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail -5 gpurun_out/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
export TMPDIR=/tmp; ROOT=$(pwd); mkdir -p gpurun_out/pmc_c2; cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex k_acc_batch -d $ROOT/gpurun_out/pmc_c2/p1 -o run --output-format csv -- python3 $ROOT/bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/pmc_c2/p1.log 2>&1 || { echo pmc failed; exit 1; }
cd $ROOT; python3 -c "
import csv,collections
v=collections.defaultdict(list)
for r in csv.DictReader(open('gpurun_out/pmc_c2/p1/run_counter_collection.csv')): v[r['Counter_Name']].append(float(r['Counter_Value']))
a={k:sum(x)/len(x) for k,x in v.items()}; print(a); print('conflict frac', a['SQ_LDS_BANK_CONFLICT']/a['SQ_LDS_IDX_ACTIVE'], 'lds util', a['SQ_LDS_IDX_ACTIVE']/(a['GRBM_GUI_ACTIVE']/8*256))"
