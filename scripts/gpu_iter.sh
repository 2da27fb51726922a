set -u
D=flink-cooccurrence_amd/csrc
cp $D/libcooc_hip.so $D/libcooc_hip_base.so
for V in base g2 g5 s22 s24 base; do
  cp $D/libcooc_hip_$V.so $D/libcooc_hip.so
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$V.json 2> gpurun_out/ab_$V.err || { tail -5 gpurun_out/ab_$V.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$V.json'));print('$V',d['ms_per_step'],d['roofline']['kernel_ms'])"
done
