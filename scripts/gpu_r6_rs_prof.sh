#!/bin/bash
# C5 owner unit (bench.py --config c5): kernel stats, the full-scoring timing, and PMC passes of the full-scoring
# k_rescore (COOC_RS_NO_NAN_EXIT=1: every entry scored).  One counter group per run, each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r6_rs
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "bench failed"; exit 1; }
COOC_RS_NO_NAN_EXIT=1 timeout -k 10 300 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5_full.json 2> $OUT/bench_c5_full.err || { echo "bench full failed"; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 "$ROOT/bench.py" --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/stats.log 2>&1 || { echo "stats failed"; exit 1; }
export COOC_RS_NO_NAN_EXIT=1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex k_rescore -d "$OUT/pmc/p$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
echo done
