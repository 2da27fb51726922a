#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/pmc_counter_collection.csv) of the dominant
kernel into profiles/pmc_accumulate.json (per-launch HBM traffic for bench.py's roofline).

Units and gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are KB;
FETCH_SIZE reports half the bytes of coalesced streaming reads on gfx950 (128-B requests tallied as
64 B), so the read side is doubled; WRITE_SIZE is taken as is."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_k_acc_batch.json"
# argv[3] = steps per pass: the counters of every matched launch of a pass summed and divided by the steps
# (several kernels per step, e.g. the counting span's k_sp_main launches + k_sp_small); else one kernel,
# averaged over its launches
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0
vals = collections.defaultdict(list)
names = set()
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        names.add((__import__("re").search(r"(k_\w+)", r["Kernel_Name"]) or [None, r["Kernel_Name"]])[1])
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
if steps:
    avg = {k: sum(v) / steps for k, v in vals.items()}  # (every counter's pass ran `steps` steps)
    res = {"kernel": "+".join(sorted(names)), "kernels": sorted(names), "per": f"step (sum of the kernels' launches, {steps} steps per pass)",
           "counters_avg": avg}
else:
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    res = {"kernel": sorted(names)[0] if names else None, "launches_averaged": max(len(v) for v in vals.values()),
           "counters_avg": avg}
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    fetch = avg["FETCH_SIZE"] * 1024
    write = avg["WRITE_SIZE"] * 1024
    res["fetch_bytes_raw"] = fetch
    res["write_bytes"] = write
    res["hbm_bytes_per_launch"] = 2 * fetch + write
    res["note"] = ("hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (KB -> B). The x2 read correction is the guide's for "
                   "wide coalesced reads (k_acc_batch reads partner ids 16 B per lane). FETCH_SIZE counts "
                   "memory-side requests (Infinity-Cache hits included): an upper bound on DRAM bytes.")
if "TCC_HIT_sum" in avg:
    res["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
if "SQ_LDS_IDX_ACTIVE" in avg and "GRBM_GUI_ACTIVE" in avg:
    res["lds_util"] = avg["SQ_LDS_IDX_ACTIVE"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 256)
    res["lds_bank_conflict_frac"] = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]
if "SQ_INSTS_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
    # VALU wave-instructions issued per SIMD-cycle (1,024 SIMDs; GRBM_GUI_ACTIVE summed over the 8 XCDs)
    res["valu_busy"] = avg["SQ_INSTS_VALU"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 1024)
if "SQ_WAIT_ANY" in avg:
    res["wave_wait_frac"] = avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
# the code the counters belong to: bench.py reports traffic / limiter only when its own source digest matches
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import source_digest  # noqa: E402

res["source_digest"] = source_digest()
sha_file = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), ".build_sha")
res["git_sha"] = open(sha_file).read().strip() if os.path.exists(sha_file) else None
os.makedirs(os.path.dirname(out), exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "counters_avg"}, indent=1))
