#!/bin/bash
# PMC passes of the C2 dense kernel (k_acc_batch) on bench.py --config c2 (two steps); one counter group
# per run, each with its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_c2
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex k_acc_batch -d "$OUT/p$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config c2 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
