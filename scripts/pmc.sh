#!/bin/bash
# PMC passes over the dominant kernel (one counter group per rocprofv3 run, no tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
GROUPS_FILE="$ROOT/${PMC_FILE:-scripts/pmc_groups.txt}"
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
done < "$GROUPS_FILE"
echo done
