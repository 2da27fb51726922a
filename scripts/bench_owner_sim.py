#!/usr/bin/env python3
"""One-GPU estimate of an owner's work in an N-GPU records run (bench.py --gpus N, weak scaling).

Every rank holds a C2-shaped shard; the owner of rows a = 0 mod N receives the records of those rows
from all N sources.  Here the N sources are the same C2 shard planned once (statistically the shape
of N shards), the collectives are replaced by slicing, and the phases are timed with HIP events:
shard_plan (each rank's local planner), shard_count (owner-side reorder + chunk plan + accumulate).
The exchange itself (RCCL over xGMI) is not measured here."""
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
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen, sharding

    W = args.parts
    d = datagen.config_c2(seed=2)
    up_h, it_h, M = d["user_ptr"], d["items"], d["n_items"]
    U, N = len(up_h) - 1, len(it_h)
    dev = torch.device("cuda", 0)
    up, it = torch.from_numpy(up_h).to(dev), torch.from_numpy(it_h).to(dev)
    core = pkg.CooccurrenceCore(n_items=M, device=0)
    core.set_kernel_timing(True)
    stride = core.shard_arena_cap(U, N)
    desc = torch.empty(N, dtype=torch.int64, device=dev)
    rc = torch.empty(M, dtype=torch.int32, device=dev)
    arena = torch.empty(stride, dtype=torch.int16, device=dev)

    def plan():
        return core.shard_plan(up, it, W, desc, rc, arena)

    for _ in range(2):
        send, ids, obs = plan()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        send, ids, obs = plan()
    torch.cuda.synchronize()
    plan_ms = (time.perf_counter() - t0) / args.steps * 1e3
    R = sharding.rows_owned(M, W, 0)
    seg = desc[:int(send[0])]
    recv_desc = torch.cat([seg] * W)
    recv_rc = torch.cat([rc[:R]] * W)
    arena_all = torch.cat([arena] * W)
    for _ in range(2):
        core.shard_count(W, 0, recv_rc, recv_desc, arena_all, stride)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ks = []
    for _ in range(args.steps):
        res = core.shard_count(W, 0, recv_rc, recv_desc, arena_all, stride)
        ks.append(core.last_kernel_ms())
    torch.cuda.synchronize()
    count_ms = (time.perf_counter() - t0) / args.steps * 1e3
    print(json.dumps({
        "parts": W, "shard": "C2 (seed 2) replicated as every source", "plan_ms": plan_ms,
        "owner_count_ms": count_ms, "owner_kernel_ms": float(np.mean(ks)), "owner_rows": R,
        "owner_pairs": int(res.observed), "owner_records": int(recv_desc.numel()),
        "arena_all_mb": arena_all.numel() * 2 / 1e6, "desc_sent_mb": desc.numel() * 8 / 1e6,
        "owner_pairs_per_s": res.observed / (count_ms * 1e-3)}))


if __name__ == "__main__":
    main()
