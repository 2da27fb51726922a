#!/usr/bin/env python3
"""Benchmark: item-pair co-occurrences counted per second on MI355X (BASELINE.json metric).

A step = one pass of the hot path over one window of synthetic input already resident in HBM:
pair expansion + keyed (itemA, itemB) count reduction + row sums (cooc_count_device), from the
CSR of user histories to the final counts in HBM.  Workload at N=1: BASELINE configs[1], the
MovieLens-20M-shaped log (138,493 users x 26,744 items, 20,000,263 interactions), numpy PCG64
seed 2.  With --gpus N (one process per GPU, torchrun), every rank expands its own C2-shaped
user shard (seed 2 + rank): users are independent units, so the per-GPU work is fixed ("weak").

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel (k_acc_batch, timed with
HIP events on the stream it runs on) and a CPU baseline (the oracle's record-by-record
restatement of the reference path, timed on a bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes(P: int, N: int, U: int, D: int) -> int:
    """4 B per ordered pair (partner id read), CSR items + offsets once, 12 B per
    distinct output key."""
    return 4 * P + 4 * N + 8 * (U + 1) + 12 * D


def cpu_baseline(user_ptr: np.ndarray, items: np.ndarray, budget_pairs: int = 80_000_000) -> dict:
    """The oracle's record-by-record restatement (NonSampled...java:113-165 -> ItemRowAggregator ->
    RowSumAggregator, one window) on the first users of the workload, ~10-20 s of one core."""
    from oracle import oracle

    n = np.diff(user_ptr)
    cum = np.cumsum(n * (n - 1))
    nu = int(np.searchsorted(cum, budget_pairs)) + 1
    sub_up = user_ptr[: nu + 1]
    sub_it = items[: sub_up[-1]]
    P = int(cum[nu - 1])
    users = np.repeat(np.arange(nu, dtype=np.int32), n[:nu])
    s = oracle.OracleStream(1000, 0)
    t0 = time.perf_counter()
    s.process_elements(users, sub_it, np.zeros(len(sub_it), np.int64))
    w = s.process_watermark(1 << 62)
    dt = time.perf_counter() - t0
    assert w and w[0].observed == P
    return {"value": P / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"first {nu} users of the same C2 log ({len(sub_it)} interactions, {P} ordered pairs), "
                      f"one window, {dt:.1f} s"}


def core_last_nnz(core) -> int:
    """Distinct keys of this rank's local (pre-exchange) result."""
    return int(core.partition_plan(1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exchange", choices=["records", "partials"], default="records",
                    help="N > 1: route pair records to owner(a) (default) or partial counts (sharding.py)")
    ap.add_argument("--pmc-file", default=os.path.join(ROOT, "profiles", "pmc_k_acc_batch.json"),
                    help="rocprofv3 PMC summary of k_acc_batch (HBM traffic per launch), if collected")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    from flink_cooccurrence_amd import sharding

    d = datagen.config_c2(seed=2 + rank)
    up_h, it_h, M = d["user_ptr"], d["items"], d["n_items"]
    U, N = len(up_h) - 1, int(up_h[-1])
    P = datagen.ordered_pairs(up_h)
    up = torch.from_numpy(up_h).to(dev)
    it = torch.from_numpy(it_h).to(dev)
    torch.cuda.synchronize()

    core = pkg.CooccurrenceCore(n_items=M, device=local_rank)
    core.set_kernel_timing(True)

    def step():
        if world == 1:
            return core.count_device(up, it)  # returns after the stream drained (errors are checked)
        # users sharded over ranks; rows owned by a mod world (keyBy(itemA), FlinkCooccurrences.java:152)
        if args.exchange == "records":
            return sharding.count_records(core, up, it)
        return sharding.count_sharded(core, up, it)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms = []
    res = None
    for _ in range(args.steps):
        res = step()
        kernel_ms.append(core.last_kernel_ms())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world == 1:
        assert res.observed == P, "pair count mismatch"
        D = int(res.nnz)
    else:
        assert res.local_observed == P, "pair count mismatch"
        D = int(res.owned.nnz) if args.exchange == "records" else int(core_last_nnz(core))

    stats = torch.tensor([elapsed, float(P), float(algorithmic_bytes(P, N, U, D))], dtype=torch.float64, device=dev)
    if world > 1:
        t = stats[:1].clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        s = stats[1:].clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        elapsed, p_total = float(t.item()), float(s[0].item())
    else:
        p_total = float(P)
    ms_per_step = elapsed / args.steps * 1e3
    value = p_total * args.steps / elapsed

    k_ms = float(np.mean(kernel_ms))
    b_alg = algorithmic_bytes(P, N, U, D)
    achieved = b_alg / (k_ms * 1e-3) / 1e9
    traffic, pmc = None, {}
    if os.path.exists(args.pmc_file):
        try:
            with open(args.pmc_file) as f:
                pmc = json.load(f)
            traffic = pmc.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic, pmc = None, {}
    out = {
        "metric": "item-pair co-occurrences counted/sec (node)",
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {
            "workload": "C2 MovieLens-20M-shaped: 138,493 users x 26,744 items, 20,000,263 interactions, "
                        "Zipf(0.9) without replacement, one window, numpy PCG64 seed 2 (+rank)",
            "users_per_gpu": U, "items": M, "interactions_per_gpu": N, "ordered_pairs_per_gpu": P,
            "distinct_keys_per_gpu": D,
            "output": "dense uint32 [items x items] in HBM" if world == 1 and res.dense else "padded CSR in HBM",
            "parallelism": f"users sharded over {world} GPU(s)" + (
                f"; rows owned by a mod N, exchange over RCCL: {args.exchange}" if world > 1 else ""),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_acc_batch",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            "traffic_gbps": (traffic / (k_ms * 1e-3) / 1e9) if traffic else None,
            "lds_util": pmc.get("lds_util"),
            "lds_bank_conflict_frac": pmc.get("lds_bank_conflict_frac"),
            "kernel_ms": k_ms,
            "algorithmic_bytes_per_launch": b_alg,
            "note": "B_alg = 4P + 4N + 8(U+1) + 12D (SURVEY.md §8(d)). frac > 1 flags cache reuse: every "
                    "partner-id list is re-read once per item in it from L2 / Infinity Cache (2 B per id "
                    "here). traffic = HBM-side bytes per launch from rocprofv3 PMC (2*FETCH_SIZE + "
                    "WRITE_SIZE, profiles/pmc_k_acc_batch.json); the kernel is bound by LDS atomics "
                    "(lds_util, lds_bank_conflict_frac), see DESIGN.md §4",
        },
        "cpu_baseline": None,
    }
    if world > 1 and args.exchange == "records":
        out["config"]["exchange"] = {
            "mode": "pair records to owner(a) = a mod N: all-gather of u16 histories + all-to-all of 8-B "
                    "descriptors; owners reduce complete rows (no partial counts, no merge)",
            "records_sent_rank0": res.sent_records, "records_recv_rank0": res.recv_records,
            "arena_bytes_per_rank": 2 * res.arena_stride, "global_ordered_pairs_per_step": res.observed}
    elif world > 1:
        out["config"]["exchange"] = {"mode": "partial rows to owner(a) = a mod N, owner merge",
                                     "entries_sent_rank0": res.sent_entries, "entries_recv_rank0": res.recv_entries,
                                     "bytes_per_entry": 8, "global_ordered_pairs_per_step": res.observed}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(up_h, it_h)
    if rank == 0:
        print(json.dumps(out), flush=True)
    core.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
