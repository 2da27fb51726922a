set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
for u in ${UNROLLS:-16 32}; do
  COOC_ACC_UNROLL=$u timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_u$u.json 2> gpurun_out/bench_u$u.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_u$u.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_u$u.json')); r=d['roofline']
print('u$u', '%.3e pairs/s'%d['value'], '%.2f ms/step'%d['ms_per_step'], 'kernel %.2f ms'%r['kernel_ms'], 'frac %.3f'%r['frac'])"
done
