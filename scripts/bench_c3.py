#!/usr/bin/env python3
"""C3 shard on one MI355X: a 1/n_shards user shard of the Zipf 1B log (1e6 items, Zipf(1.0) with
replacement, lognormal lengths of mean 100 capped at 10,000; datagen.config_c3), counted with
cooc_count_device.  n_items = 1e6 > 40,320, so this is the column-tiled general planner with the
sparse padded-CSR output, not the C2 batch planner.

Prints one JSON line per shard count: median device time (HIP events around the whole call, inputs
resident in HBM), pairs/s, the nnz of the result, and the size-independent checks
sum(rowsum) == observed == P (P from the generator).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=64, help="C3 is split into this many user shards; shard 0 runs")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen

    t0 = time.perf_counter()
    d = datagen.config_c3(shard=0, n_shards=args.shards)
    up_h, it_h, M = d["user_ptr"], d["items"], d["n_items"]
    P = datagen.ordered_pairs(up_h)
    t_gen = time.perf_counter() - t0
    dev = torch.device("cuda", 0)
    up, it = torch.from_numpy(up_h).to(dev), torch.from_numpy(it_h).to(dev)
    core = pkg.CooccurrenceCore(n_items=M, device=0)
    res = core.count_device(up, it)  # warm-up (allocations)
    torch.cuda.synchronize()
    times = []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        res = core.count_device(up, it)  # synchronises the context's stream before it returns
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    rowsum = torch.zeros(M, dtype=torch.int64, device=dev)
    core.copy_rowsum_device(rowsum)
    torch.cuda.synchronize()
    rs_total = int(rowsum.sum().item())
    ms = float(np.median(times))
    out = {
        "config": d["name"],
        "users": int(len(up_h) - 1),
        "interactions": int(it_h.size),
        "items": int(M),
        "ordered_pairs": int(P),
        "nnz": int(res.nnz),
        "ms": ms,
        "ms_all": times,
        "pairs_per_s": P / (ms * 1e-3),
        "check_observed_eq_P": int(res.observed) == P,
        "check_sum_rowsum_eq_P": rs_total == P,
        "gen_s": t_gen,
    }
    print(json.dumps(out), flush=True)
    core.close()
    if not (out["check_observed_eq_P"] and out["check_sum_rowsum_eq_P"]):
        sys.exit(1)


if __name__ == "__main__":
    main()
