set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
bash scripts/pmc_rescore.sh || exit 1
python scripts/pmc_summary.py gpurun_out/pmc_rs gpurun_out/pmc_k_rescore.json > /dev/null; python -c "
import json; d=json.load(open('gpurun_out/pmc_k_rescore.json')); c=d.pop('counters_avg'); print(d); g=c['GRBM_GUI_ACTIVE']; print('valu/cu-cycle', c['SQ_INSTS_VALU']/(g/8*256), 'vmem rd', c['SQ_INSTS_VMEM_RD'], 'lat', c['TCP_TCC_READ_REQ_LATENCY_sum']/c['TCP_TCC_READ_REQ_sum'])"
