set -u
mkdir -p gpurun_out/perm
for p in "" "--permute"; do
  n=rank; [ -n "$p" ] && n=perm
  timeout -k 10 300 python -u scripts/bench_c3.py --steps 3 $p > gpurun_out/perm/bench_$n.json 2> gpurun_out/perm/bench_$n.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/perm/bench_$n.json'));print('$n', 'ms', round(d['ms'],2), 'k_sp_main', round(d['k_sp_main_ms'],2), 'nnz', d['nnz'], d['verify'])"
  timeout -k 10 300 python -u scripts/bench_c3.py --steps 2 $p --lib flink-cooccurrence_amd/csrc/libcooc_hip_stats.so > gpurun_out/perm/stats_$n.txt 2>&1 || exit 1
  grep "sp stats" gpurun_out/perm/stats_$n.txt | tail -8
done
