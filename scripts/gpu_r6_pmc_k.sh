#!/bin/bash
# PMC passes (one counter group per run, each under its own limit) of the kernels matching $KREGEX in the C5 owner
# unit (bench.py --config c5, one step), summarised by scripts/pmc_summary.py into $OUT/summary.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
KREGEX=${KREGEX:-k_rs_score}
OUT=$ROOT/gpurun_out/${PMC_TAG:-pmc_k}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex "$KREGEX" -d "$OUT/pmc/p$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmc_p$i.log"; exit 1; }
  echo "pass $i ok"
done
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT/pmc" "$OUT/summary.json" ${PMC_STEPS:-} && rm -rf "$OUT/pmc" && cat "$OUT/summary.json"
