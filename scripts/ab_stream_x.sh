# A/B of k_acc_batch experiment modes on the C4 stream (COOC_ACC_X: 0 full, 4 no walk, 8 no stores,
# 20 neither walk nor compaction)
set -e
mkdir -p gpurun_out/xab
export TMPDIR=/tmp
for X in ${XS:-0 4 8}; do
  COOC_ACC_X=$X timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xab/x$X -o run -- python3 scripts/bench_stream.py --windows ${WINDOWS:-30} > gpurun_out/xab/x$X.log 2>&1
done
