# rocprofv3 kernel stats of the C3 share, rank-ordered and permuted ids (the line's any-order flag).
set -o pipefail
export TMPDIR=/tmp COOC_BENCH_ANY_ORDER=1
R=$(pwd)
mkdir -p gpurun_out
cd /tmp
for p in "" --permute; do
  n=rank; [ -n "$p" ] && n=perm
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$n -o run --output-format csv -- python3 $R/scripts/bench_c3.py --steps 3 $p > $R/gpurun_out/prof_$n.log 2>&1 || { echo "prof $n failed"; exit 1; }
  echo "prof $n ok"
done
