# C5 rescoring timing experiments (results of the rs1/rs2/rs3 builds are invalid by construction):
# rs1 = no log in the k11 == 1 score, rs2 = no heap feeding, rs4 = no logs in the full formula (k11 != 1); bits combine.
set -o pipefail
mkdir -p gpurun_out
for v in base rs7 rs8 rs15 rs31; do
  if [ $v = base ]; then unset COOC_LIB; else export COOC_LIB=flink-cooccurrence_amd/csrc/libcooc_hip_$v.so; fi
  timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-permuted > gpurun_out/c5x_$v.json 2> gpurun_out/c5x_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/c5x_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c5x_$v.json'));r=d.get('roofline_rescore',{});print('$v', 'ms', round(d['ms_per_step'],2), 'rescore ms', round(r.get('kernel_ms'),2))"
done
