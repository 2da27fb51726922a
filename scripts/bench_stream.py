#!/usr/bin/env python3
"""C4 (BASELINE configs[3]): streaming tumbling windows into resident device state.

The C2 log with event times spread over 100 tumbling 1 s windows (seed 4).  Every window is staged
with cooc_submit_batch (users and their new items, arrival order) and processed by
cooc_finish_window: expansion against the resident histories, the window's delta rows and row
sums, the merge into the resident dense global rows and, with --topk, LLR rescoring of every
touched row (the C5 stage at C2 scale).  Reports per-window latency and incremental pairs/s; the
copy of each window's outputs to the host (what a Flink operator would emit) is timed separately.
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
    ap.add_argument("--windows", type=int, default=100)
    ap.add_argument("--topk", type=int, default=0)
    ap.add_argument("--copy", action="store_true", help="also copy every window's outputs to the host")
    ap.add_argument("--users", type=int, default=138_493)
    ap.add_argument("--planner", default="auto", choices=["auto", "large", "general", "sort"])
    ap.add_argument("--c3-shard", type=int, default=0,
                    help="stream users [0, 1e7 / this) of the C3 log (1e6 items) instead of the C2 log")
    args = ap.parse_args()

    import torch

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen

    t0 = time.time()
    if args.c3_shard:
        up3, it3 = datagen.c3_users(0, datagen.C3_USERS // args.c3_shard)
        rng = np.random.Generator(np.random.PCG64(4))
        d = {"user_ptr": up3, "items": it3, "n_items": datagen.C3_ITEMS,
             "ts": datagen.spread_over_windows(rng, up3, args.windows, 1000)}
    elif args.users == 138_493:
        d = datagen.config_c4(n_windows=args.windows)
    else:  # reduced log (same shape) for quick runs
        N = int(20_000_263 * args.users / 138_493)
        d = datagen.config_c2(U=args.users, N=N)
        rng = np.random.Generator(np.random.PCG64(4))
        d["ts"] = datagen.spread_over_windows(rng, d["user_ptr"], args.windows, 1000)
    up, it, ts, M = d["user_ptr"], d["items"], d["ts"], d["n_items"]
    lens = np.diff(up)
    owner = np.repeat(np.arange(len(lens), dtype=np.int32), lens)
    win = ts // 1000
    gen_s = time.time() - t0
    # per-window CSR (users ascending, arrival order inside a user: ts ascending within a user already)
    order = np.lexsort((ts, owner, win))
    w_sorted, u_sorted, i_sorted = win[order], owner[order], it[order]
    bounds = np.searchsorted(w_sorted, np.arange(args.windows + 1))
    batches = []
    for w in range(args.windows):
        s, e = bounds[w], bounds[w + 1]
        uu = u_sorted[s:e]
        change = np.nonzero(np.diff(uu))[0] + 1
        starts = np.concatenate([[0], change])
        user_ids = uu[starts]
        user_ptr = np.concatenate([starts, [e - s]]).astype(np.int64)
        batches.append((w * 1000 + 999, user_ids.astype(np.int32), user_ptr, i_sorted[s:e].astype(np.int32)))

    core = pkg.CooccurrenceCore(n_items=M, topk=args.topk, window_size_ms=1000, device=0, planner=args.planner)
    lat, copy_s, pairs = [], [], []
    for ts_w, uid, uptr, items in batches:
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        core.submit_batch(ts_w, uid, uptr, items)
        info = core.finish_window_info(ts_w)
        lat.append(time.perf_counter() - t1)
        pairs.append(info.observed)
        if args.copy:
            t2 = time.perf_counter()
            core.window_result(info)
            copy_s.append(time.perf_counter() - t2)
    total_pairs = int(np.sum(pairs))
    assert total_pairs == datagen.ordered_pairs(up), "sum of window pairs != pairs of the whole log"
    lat_ms = np.array(lat) * 1e3
    out = {
        "config": "C4 streaming: %s over %d x 1 s windows (seed 4)%s" % (
            f"users [0, 1e7/{args.c3_shard}) of the C3 log (1e6 items; sparse global rows, windows as "
            "C(full) - C(old))" if args.c3_shard else "C2-shaped log",
            args.windows, f", LLR top-{args.topk} rescoring of touched rows" if args.topk else ""),
        "users": int(len(lens)), "interactions": int(up[-1]), "n_items": M,
        "windows": args.windows, "topk": args.topk, "planner": args.planner,
        "window_latency_ms": {"median": float(np.median(lat_ms)), "p90": float(np.percentile(lat_ms, 90)),
                              "max": float(lat_ms.max()), "first": float(lat_ms[0]), "last": float(lat_ms[-1])},
        "total_s": float(np.sum(lat)), "ordered_pairs": total_pairs,
        "incremental_pairs_per_s": total_pairs / float(np.sum(lat)),
        "interactions_per_s": float(up[-1]) / float(np.sum(lat)),
        "datagen_s": gen_s,
    }
    if copy_s:
        out["copy_out_ms_median"] = float(np.median(copy_s) * 1e3)
    print(json.dumps(out), flush=True)
    core.close()


if __name__ == "__main__":
    main()
