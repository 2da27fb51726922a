#!/bin/bash
# PMC passes over the dominant kernel (one counter group per rocprofv3 run, no tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
cd /tmp
i=0
while IFS= read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --kernel-include-regex "${KREGEX:-k_accumulate}" \
    -d "$ROOT/gpurun_out/pmc/p$i" -o pmc --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/pmc/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$ROOT/gpurun_out/pmc/p$i.log"; exit $rc; }
done <<GROUPS
${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE}
GROUPS
echo done
