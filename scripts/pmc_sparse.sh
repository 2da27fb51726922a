#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes of the large-universe counting kernels (the span bench.py times:
# k_sp_main's launches, k_sp_small, k_sp_tiny, k_sp_split_finalize) on one GPU's 1/8 share of C3
# (scripts/bench_c3.py, with the bench line's COOC_FLAG_ANY_ORDER; each pass runs 2 steps: warm-up + 1).
# One counter group per run (rocprofv3 does not split passes);
# every run has its own time limit and a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_sp
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
SHARDS=${SHARDS:-8}
export COOC_BENCH_ANY_ORDER=${COOC_BENCH_ANY_ORDER:-1}
KREGEX='k_sp_(main|small|tiny|split_finalize)'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$ROOT/scripts/bench_c3.py" --shards $SHARDS --steps 2 > "$OUT/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
tail -1 "$OUT/trace.log" | cut -c1-300
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "$KREGEX" -d "$OUT/p$i" -o run --output-format csv \
    -- python3 "$ROOT/scripts/bench_c3.py" --shards $SHARDS --steps 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
find "$OUT" -name "*counter_collection.csv" | head
