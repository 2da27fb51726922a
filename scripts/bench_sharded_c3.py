#!/usr/bin/env python3
"""One-GPU measurement of the north star's literal C3 exchange at N GPUs (sharding.count_sharded): every
rank counts its own users, packs its PARTIAL rows by owner (a mod N) and all-to-alls them; the owner
merges N partial rows per owned row.  DESIGN.md §5 chooses the owned-rows exchange (count_owned: the
histories all-gathered, 4 B per interaction) instead; this script measures what the partial-count
exchange would move and cost, for owner `part`:
  * per rank r (users [r U/8, (r+1) U/8) of the shard-invariant 1B log): count time, pack time and the
    bytes it sends to every owner (8 B per partial entry);
  * the owner's merge of the N received slices (cooc_merge_partitions), timed.
The all-to-all itself (RCCL over xGMI) is not run here: its bytes are reported.  Prints one JSON line."""
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
    ap.add_argument("--part", type=int, default=0, help="the owner whose merge is timed")
    ap.add_argument("--ranks", type=int, default=None, help="ranks actually counted (default: all)")
    args = ap.parse_args()
    import torch

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen, sharding

    dev = torch.device("cuda", 0)
    W, part = args.world, args.part
    U8 = datagen.C3_USERS // 8
    M = datagen.C3_ITEMS
    R = sharding.rows_owned(M, W, part)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    core = pkg.CooccurrenceCore(n_items=M, device=0)
    core.set_kernel_timing(True)
    recv_nnz, recv_ent, ranks = [], [], []
    rowsum = torch.zeros(M, dtype=torch.int64, device=dev)
    for r in range(args.ranks or W):
        up, it = datagen.c3_users(r * U8, (r + 1) * U8, device=dev)
        core.count_device(up, it)  # (warm-up / allocations)
        ev0.record()
        res = core.count_device(up, it)
        ev1.record()
        ev1.synchronize()
        count_ms = ev0.elapsed_time(ev1)
        plan = core.partition_plan(W)
        row_nnz = torch.empty(M, dtype=torch.int32, device=dev)
        entries = torch.empty(int(plan.sum()), dtype=torch.int64, device=dev)
        ev0.record()
        core.partition_pack(W, row_nnz, entries)
        ev1.record()
        ev1.synchronize()
        pack_ms = ev0.elapsed_time(ev1)
        rs = torch.empty(M, dtype=torch.int64, device=dev)
        core.copy_rowsum_device(rs)
        rowsum += rs
        # owner-major packing: owner o's rows_owned(o) row counts, then its entries
        ro = [sharding.rows_owned(M, W, o) for o in range(W)]
        r0 = sum(ro[:part])
        e0 = int(plan[:part].sum())
        recv_nnz.append(row_nnz[r0:r0 + R].clone())
        recv_ent.append(entries[e0:e0 + int(plan[part])].clone())
        ranks.append({"rank": r, "count_ms": count_ms, "k_sp_main_ms": core.last_kernel_ms(), "pack_ms": pack_ms,
                      "partial_entries": int(res.nnz), "sent_bytes": int(8 * (plan.sum() - plan[r % W])),
                      "sent_bytes_to_owner": [int(8 * x) for x in plan]})
        del up, it, row_nnz, entries, rs
        torch.cuda.empty_cache()
    nnz_all = torch.cat(recv_nnz)
    ent_all = torch.cat(recv_ent)
    del recv_nnz, recv_ent
    torch.cuda.empty_cache()
    # the owner's merge: cooc_merge_partitions keeps a dense LDS row per owned row (n_items < 40,320); at
    # 1e6 items the N partial rows of a row would be merged by sorting the received (row, column) keys and
    # reducing equal keys -- timed here on a 1e9-entry slice of the received entries with torch.sort
    # (the dominant step), then scaled to all of them
    merge_ms, merged_nnz = [None], None
    if M <= 40_704:
        merge_ms = []
        for _ in range(2):
            ev0.record()
            merged = core.merge_partitions(W, part, nnz_all, ent_all, rowsum_global=rowsum)
            ev1.record()
            ev1.synchronize()
            merge_ms.append(ev0.elapsed_time(ev1))
        merged_nnz = int(merged.nnz)
    n_sl = min(int(ent_all.numel()), 1_000_000_000)
    rows_of = torch.repeat_interleave(torch.arange(W * R, device=dev, dtype=torch.int64) % R, nnz_all.to(torch.int64))
    keys = (rows_of[:n_sl] << 32) | (ent_all[:n_sl] >> 32)
    del rows_of
    torch.cuda.synchronize()
    ev0.record()
    torch.sort(keys)
    ev1.record()
    ev1.synchronize()
    sort_ms = ev0.elapsed_time(ev1)
    out = {"config": f"C3 partial-count exchange at N={W}: ranks' 1/8 user shares of the shard-invariant 1B log, "
                     f"owner {part} ({R} rows owned)",
           "ranks": ranks, "owner_recv_entries": int(ent_all.numel()), "owner_recv_bytes": int(8 * ent_all.numel()),
           "owner_merge_ms": merge_ms[-1], "owner_merged_entries": merged_nnz,
           "merge_sort_proxy": {"entries_sorted": n_sl, "ms": sort_ms,
                                "ms_scaled_to_all_received": sort_ms * ent_all.numel() / n_sl},
           "owned_rows_exchange_bytes_per_rank": 4 * 999_536_273 * (W - 1) // W,
           "note": "sent_bytes = 8 B x the rank's partial entries owned elsewhere (what the all-to-all moves out "
                   "of one rank); owned_rows_exchange_bytes_per_rank = what count_owned's all-gather moves in"}
    print(json.dumps(out), flush=True)
    core.close()


if __name__ == "__main__":
    main()
