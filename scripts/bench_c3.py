#!/usr/bin/env python3
"""C3 shard on one MI355X: users [0, 1e7 / shards) of the shard-invariant Zipf 1B log
(datagen.c3_users: 1e6 items, Zipf(1.0) with replacement, lognormal lengths of mean 100), generated on
the GPU and counted with cooc_count_device (n_items = 1e6: the large-universe path, cooc_sparse.hip).

Prints one JSON line: median time of the whole call (HIP events on the stream it runs on, inputs
resident in HBM), the k_sp_main time, pairs/s, the nnz of the result, and the size-independent
checks observed == P and sum(rowsum) == P (P from the generator's lengths).
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
    ap.add_argument("--shards", type=int, default=8, help="C3 users / this many are counted (8: one GPU's share)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--lib", default=None, help="another build of libcooc_hip.so (e.g. the statistics build)")
    ap.add_argument("--planner", default="auto", help='CooccurrenceCore planner ("sort": every whole row through '
                    'the sort + segmented-reduce path)')
    ap.add_argument("--permute", action="store_true", help="item ids through datagen.c3_item_perm (not rank-ordered)")
    ap.add_argument("--n-items", type=int, default=None, help="the universe passed to the core (default 1e6; "
                    "larger: unused items at the top, more tiles)")
    ap.add_argument("--column-order", action="store_true", help="COOC_FLAG_COLUMN_ORDER (no frequency relabel)")
    args = ap.parse_args()
    import torch

    import __graft_entry__


    pkg = __graft_entry__.load_package()
    if args.lib:  # before the first call loads the library
        sys.modules["flink_cooccurrence_amd._lib"].LIB_PATH = os.path.abspath(args.lib)
    from flink_cooccurrence_amd import datagen

    dev = torch.device("cuda", 0)
    U = datagen.C3_USERS // args.shards
    t0 = time.perf_counter()
    up, it = datagen.c3_users(0, U, device=dev, permute=args.permute)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    P = datagen.c3_ordered_pairs(0, U)
    M = args.n_items or datagen.C3_ITEMS
    # COOC_BENCH_ANY_ORDER=1: COOC_FLAG_ANY_ORDER (rows in no particular order; A/B through the environment)
    any_order = os.environ.get("COOC_BENCH_ANY_ORDER", "0") == "1"
    core = pkg.CooccurrenceCore(n_items=M, device=0, planner=args.planner, column_order=args.column_order,
                                any_order=any_order)
    core.set_kernel_timing(True)
    res = core.count_device(up, it)  # warm-up (allocations)
    torch.cuda.synchronize()
    times, kms = [], []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        res = core.count_device(up, it)  # on torch's current stream; returns after it drained
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
        kms.append(core.last_kernel_ms())
    rowsum = torch.zeros(M, dtype=torch.int64, device=dev)
    core.copy_rowsum_device(rowsum)
    torch.cuda.synchronize()
    rs_total = int(rowsum.sum().item())
    ms = float(np.median(times))
    out = {
        "config": f"C3 shard-invariant log, users [0, {U}) (1/{args.shards} of 1e7), 1e6 items",
        "users": U,
        "interactions": int(it.numel()),
        "items": M,
        "ordered_pairs": P,
        "nnz": int(res.nnz),
        "ms": ms,
        "ms_all": times,
        "k_sp_main_ms": float(np.median(kms)),
        "pairs_per_s": P / (ms * 1e-3),
        "check_observed_eq_P": int(res.observed) == P,
        "check_sum_rowsum_eq_P": rs_total == P,
        "gen_s": t_gen,
        "planner": args.planner,
        "permuted_ids": args.permute,
        "column_order": args.column_order,
        "sort_path_rows_pairs": core.last_sort_rows(),
        "verify": core.verify_batch(),
    }
    print(json.dumps(out), flush=True)
    core.close()
    if not (out["check_observed_eq_P"] and out["check_sum_rowsum_eq_P"]):
        sys.exit(1)


if __name__ == "__main__":
    main()
