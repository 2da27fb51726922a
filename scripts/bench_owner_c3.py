#!/usr/bin/env python3
"""One-GPU estimate of a rank's compute in the N-GPU C3 run (bench.py --gpus N: sharding.count_owned).

At N GPUs every rank all-gathers the whole log's histories and counts the rows it owns over all of
them (cooc_count_device_owned).  Here the whole shard-invariant C3 log of N x 1.25e6 users is built on
one GPU (the state after the all-gather), the owner map is the same snake_owner of the global item
frequencies, and rank `part`'s counting step is timed (HIP events on its stream).  The exchange itself
(RCCL all-gather over xGMI) is not measured here.  Prints one JSON line."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--parts", default="0", help="comma-separated ranks to time")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--permute", action="store_true", help="item ids permuted (datagen.c3_item_perm)")
    ap.add_argument("--lib", default=None, help="another build of libcooc_hip.so")
    args = ap.parse_args()
    import torch

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    if args.lib:  # before the first call loads the library
        sys.modules["flink_cooccurrence_amd._lib"].LIB_PATH = os.path.abspath(args.lib)
    from flink_cooccurrence_amd import datagen, sharding

    dev = torch.device("cuda", 0)
    U8 = datagen.C3_USERS // 8
    ups, its = [], []
    base = 0
    for r in range(args.world):
        up, it = datagen.c3_users(r * U8, (r + 1) * U8, device=dev, permute=args.permute)
        ups.append(up[:-1] + base)
        its.append(it)
        base += int(up[-1].item())
        del up
    up = torch.cat(ups + [torch.tensor([base], dtype=torch.int64, device=dev)])
    it = torch.cat(its)
    del ups, its
    M = datagen.C3_ITEMS
    N = int(it.numel())
    # (COOC_BENCH_ANY_ORDER=1: the bench line's COOC_FLAG_ANY_ORDER)
    core = pkg.CooccurrenceCore(n_items=M, device=0, any_order=os.environ.get("COOC_BENCH_ANY_ORDER", "0") == "1")
    core.set_kernel_timing(True)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # the rank's own share of the frequencies (cooc_item_counts on 1/world of the log), timed
    core.item_counts(it[: N // args.world])
    ev0.record()
    core.item_counts(it[: N // args.world])
    ev1.record()
    ev1.synchronize()
    freq_ms = ev0.elapsed_time(ev1)
    freq = core.item_counts(it)
    owner = sharding.snake_owner(freq, args.world)
    out = {"config": f"C3 rank compute at N={args.world}: all {args.world * U8} users ({N} interactions) after the "
                     f"all-gather, rows owned by snake_owner(freq, {args.world})", "permuted_ids": args.permute,
           "parts": {}}
    P_all = 0
    for part in [int(x) for x in args.parts.split(",")]:
        ms, kms = [], []
        for s in range(args.steps + 1):
            ev0.record()
            res = core.count_device_owned(up, it, owner, part, freq, N)
            ev1.record()
            ev1.synchronize()
            if s:
                ms.append(ev0.elapsed_time(ev1))
                kms.append(core.last_kernel_ms())
        P_all += int(res.observed)
        out["parts"][part] = {"ms": float(np.median(ms)), "k_sp_main_ms": float(np.median(kms)),
                              "outside_counting_span_ms": float(np.median(ms)) - float(np.median(kms)),
                              "ordered_pairs": int(res.observed), "nnz": int(res.nnz),
                              "pairs_per_s": int(res.observed) / (float(np.median(ms)) * 1e-3)}
    out["interactions"] = N
    out["item_counts_ms_per_rank_share"] = freq_ms
    # the all-gather each rank would run first (not measured here): the other ranks' item ids (4 B each) and
    # user pointers (8 B per user), modelled over xGMI at LINK_GBPS per link (MI355X: 7 links per GPU in an
    # 8-GPU node) -- received from all 7 peers at once (direct / mesh) or one link per step (ring)
    link_gbps = float(os.environ.get("LINK_GBPS", "153"))
    recv = (N - N // args.world) * 4 + (args.world * U8 - U8) * 8
    out["allgather_model"] = {"bytes_received_per_rank": recv, "link_GBps": link_gbps,
                              "mesh_ms": recv / (min(7, args.world - 1) * link_gbps * 1e9) * 1e3,
                              "ring_ms": recv / (link_gbps * 1e9) * 1e3,
                              "note": "modelled, not measured: bytes / bandwidth, no latency or protocol overhead"}
    print(json.dumps(out), flush=True)
    core.close()


if __name__ == "__main__":
    main()
