#!/bin/bash
# Instruction-fetch PMC of the counting kernels (k_sp_main's two shapes, k_sp_small) on one GPU's 1/8 share of
# C3 (scripts/bench_c3.py): instruction-cache hits / misses, instruction fetches, the waves' instruction-wait
# cycles.  One counter group per run, each under its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_ic
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES" \
           "SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "k_sp_main|k_sp_small" -d "$OUT/p$i" -o run \
    --output-format csv -- python3 "$ROOT/scripts/bench_c3.py" --steps 1 ${PMC_ARGS:-} > "$OUT/p$i.log" 2>&1 \
    || { echo "pass $i failed"; tail -3 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k][r["Counter_Name"]] += 1
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {v:.4g}")
PY
