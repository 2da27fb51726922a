#!/usr/bin/env python3
"""Benchmark: item-pair co-occurrences counted per second on MI355X (BASELINE.json metric).

A step = one pass of the hot path over one window of synthetic input already resident in HBM: pair
expansion + keyed (itemA, itemB) count reduction + row sums, from the CSR of user histories to the
final counts in HBM (padded CSR).

Workload (default --config c3): the north star's Zipf-skewed 1B log (BASELINE configs[2]: 1e7
users x 1e6 items, 1e9 interactions), generated shard-invariantly (datagen.c3_users: every user's
list is a function of (seed, user id)) directly on each GPU.  Rank r of N holds users
[r U/8, (r+1) U/8): per-GPU work is fixed ("weak" scaling) and at N = 8 the ranks hold the whole
1B log.  N = 1 therefore runs one GPU's 1/8 share of C3 (1.25e6 users, 1.25e8 interactions,
3.36e10 ordered pairs).  N > 1: the ranks all-gather the histories over RCCL and each counts the
rows it owns (sharding.count_owned, the keyBy(itemA) of FlinkCooccurrences.java:152); the
all-gather, the item-frequency all-reduce and the owner map are inside the timed step.
--config c2: the MovieLens-20M-shaped log (configs[1]) per rank, records exchange for N > 1.
--config c5 (configs[4], LLR + per-item top-k): at N = 1 the unit one rank of the 8-GPU job computes -- the whole
1B log resident (the state after the histories' all-gather), the rows rank --c5-part owns under the snake owner map
of the whole log's item frequencies counted over every user (cooc_count_device_owned), then every owned row scored
against the WHOLE log's row sums and observed total (what the row-sum all-reduce hands every owner) and its top-k
kept (cooc_topk_batch_device).  N > 1: the same through the library's exchange (sharding.count_owned / topk_owned).

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel (HIP events on the stream
it runs on) and a CPU baseline (the oracle's multithreaded record-by-record restatement on a
bounded sample of the same log, all the host threads of this GPU's share).
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
LDS_ADD_PEAK = 6.89 * 256 * 2.4e9  # random-slot no-return ds_add lane-ops/s, measured (profiles/r02/micro/lds_atomics.txt)
METRIC = "item-pair co-occurrences counted/sec (node) at 1/2/4/8 GPUs; achieved HBM GB/s"


def algorithmic_bytes(P: int, N: int, U: int, D: int) -> int:
    """4 B per ordered pair (partner id read), CSR items + offsets once, 12 B per
    distinct output key."""
    return 4 * P + 4 * N + 8 * (U + 1) + 12 * D


def cpu_baseline(user_ptr: np.ndarray, items: np.ndarray, n_items: int, what: str, target_s: float = 20.0,
                 threads_override: int = 0) -> dict:
    """The oracle's multithreaded record-by-record restatement (threads own rows a mod T, every
    thread expands every user's records, NonSampled...java:129-161 -> ItemRowAggregator addTo) on
    the first users of the same log: a calibration run sizes the sample (its small size underestimates the
    rate, so a target of 20 s gives a run of ~10-15 s)."""
    from oracle import oracle

    threads, nproc, avail = cpu_threads()
    if threads_override > 0:
        threads = threads_override
    n = np.diff(user_ptr)
    cum = np.cumsum(n * (n - 1))

    def sample(pairs: int):
        nu = min(len(n), int(np.searchsorted(cum, pairs)) + 1)
        up = user_ptr[: nu + 1]
        return nu, up, items[: up[-1]]

    nu, up, it = sample(20_000_000)
    t0 = time.perf_counter()
    oracle.count_batch_mt(up, it, n_items, threads)
    rate = max(1.0, float(cum[nu - 1]) / (time.perf_counter() - t0))
    nu, up, it = sample(int(min(2.5e9, rate * target_s)))  # (~10-15 s on the GPU box host; RAM ~30 GB)
    P = int(cum[nu - 1])
    t0 = time.perf_counter()
    nnz, pairs = oracle.count_batch_mt(up, it, n_items, threads)
    dt = time.perf_counter() - t0
    assert pairs == P
    return {"value": P / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "nproc": nproc, "cpus_available": avail,
            "threads_rule": ("the GPU box's CPU share per GPU (OMP_NUM_THREADS; the affinity mask lists the whole host's "
                             "CPUs, shared by the node's GPUs); bench.py --cpu-threads N times another count"
                             if not threads_override else "--cpu-threads"),
            "label": "CPU restatement, not the JVM reference (BASELINE.md)",
            # the figure for every CPU in the affinity mask, by linear scaling of the measured one (an upper bound:
            # the restatement is memory-bound and shares the host with the node's other GPUs' processes); not timed
            "all_cpus_linear_upper_bound": {"value": P / dt * avail / threads, "cpus": avail, "measured": False},
            "sample": f"first {nu} users of {what} ({len(it)} interactions, {P} ordered pairs, {nnz} keys), "
                      f"one window, {threads} threads, {dt:.1f} s"}


def cpu_threads():
    """Threads for the CPU baseline: every CPU this process may run on (nproc), capped by
    OMP_NUM_THREADS when the environment sets it (the GPU box sets it to its CPU share per GPU).
    Returns (threads, nproc, CPUs in the affinity mask)."""
    nproc = os.cpu_count() or 1
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(avail, cap) if cap > 0 else avail), nproc, avail


def source_digest() -> str:
    """sha256 over the library's kernel and host sources (csrc/*.hip, *.cpp, *.h, Makefile): ties a
    profiles/pmc_<kernel>.json to the code it was collected on (scripts/pmc_summary.py records it)."""
    import hashlib

    d = os.path.join(ROOT, "flink-cooccurrence_amd", "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".cpp", ".h")) or f == "Makefile":
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


def entries_read(res, M: int, k: int, sizes, scores):
    """Entries k_rescore reads (cooc_stream.hip): every entry of a row, except that a row whose heap is full
    with a NaN root stops after its first ceil(k / 64) * 64 entries (min 512)."""
    import ctypes

    import torch

    nnz = np.zeros(M, np.int32)
    hip = ctypes.CDLL("libamdhip64.so")
    if hip.hipMemcpy(nnz.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(res.row_nnz), ctypes.c_size_t(nnz.nbytes),
                     ctypes.c_int(2)) != 0:
        return None
    first = min(512, (k + 63) // 64 * 64)
    cut = ((sizes == k) & torch.isnan(scores[:, 0])).cpu().numpy()
    n = nnz.astype(np.int64)
    return int(np.where(cut, np.minimum(n, first), n).sum())


def limiter(pmc: dict, traffic, k_ms: float):
    """What the PMC counters (profiles/pmc_<kernel>.json, collected by scripts/pmc_sparse.sh) say
    bounds the kernel: HBM when the measured HBM-side bytes run near the peak, LDS when the LDS is
    busy most cycles, else memory latency (waves waiting on outstanding loads with both far from
    their peaks)."""
    if not pmc or not traffic:
        return None
    hbm = traffic / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
    lds = pmc.get("lds_util") or 0.0
    wait = pmc.get("wave_wait_frac") or 0.0
    if hbm >= 0.7:
        kind = "hbm"
    elif lds >= 0.6:
        kind = "lds"
    else:
        kind = "latency"
    return (f"{kind}: measured HBM traffic at {hbm:.0%} of peak, LDS busy {lds:.0%} of cycles, waves waiting "
            f"{wait:.0%} of their cycles (PMC of the same kernel, profiles/pmc_{pmc.get('kernel', 'kernel')}.json)")


def load_pmc(path: str) -> dict:
    if os.path.exists(path):
        try:
            with open(path) as f:
                return json.load(f)
        except (OSError, ValueError):
            return {}
    return {}


def c4_batches(n_windows: int = 100):
    """BASELINE configs[3]: the C2 log with event times over n_windows tumbling 1 s windows (datagen.config_c4,
    seed 4) as per-window batches (window maxTimestamp, user ids, user_ptr, items; users ascending, each user's
    new items in arrival order) -- what GpuNonSampledCooccurrenceRowsOperator hands cooc_submit_batch."""
    from flink_cooccurrence_amd import datagen

    d = datagen.config_c4(n_windows=n_windows)
    up, it, ts, M = d["user_ptr"], d["items"], d["ts"], d["n_items"]
    lens = np.diff(up)
    owner = np.repeat(np.arange(len(lens), dtype=np.int32), lens)
    win = ts // 1000
    order = np.lexsort((ts, owner, win))
    w_sorted, u_sorted, i_sorted = win[order], owner[order], it[order]
    bounds = np.searchsorted(w_sorted, np.arange(n_windows + 1))
    batches = []
    for w in range(n_windows):
        s0, e0 = bounds[w], bounds[w + 1]
        uu = u_sorted[s0:e0]
        starts = np.concatenate([[0], np.nonzero(np.diff(uu))[0] + 1]).astype(np.int64)
        batches.append((w * 1000 + 999, uu[starts].astype(np.int32), np.concatenate([starts, [e0 - s0]]).astype(np.int64),
                        i_sorted[s0:e0].astype(np.int32)))
    return d, batches


def run_c4(args):
    """C4 (BASELINE configs[3]): streaming 1 s windows into resident device state on one GPU.  A step is one window:
    cooc_submit_batch + cooc_finish_window -- the window's pairs expanded against the users' resident histories
    (NonSampled...java:129-161), its delta rows and row sums reduced (ItemRowAggregator / RowSumAggregator), merged
    into the resident global rows and row sums and every touched row rescored, LLR top-k (ItemRowRescorer...java:
    144-228).  Warm-up: the whole stream once on a context that is then dropped; timed: the whole stream again on a
    fresh context (state from empty, as a job starts), every window bracketed by device synchronisations."""
    import torch

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--config c4 runs on one GPU (its multi-GPU streaming is tests/test_streaming_multiproc.py)")
    n_windows = 100
    d, batches = c4_batches(n_windows)
    M, topk = d["n_items"], (args.topk if args.topk != 50 else 10)  # (the reference's default topK, Configuration.java:153)
    torch.cuda.set_device(0)

    def stream(core, timed):
        lat, kms, pairs, nnz, users, inter = [], [], [], [], [], []
        for ts_w, uid, uptr, items in batches:
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            core.submit_batch(ts_w, uid, uptr, items)
            info = core.finish_window_info(ts_w)
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t1)
            if timed:
                kms.append(core.last_kernel_ms())
                pairs.append(int(info.observed))
                nnz.append(int(info.nnz))
                users.append(len(uid))
                inter.append(len(items))
        return lat, kms, pairs, nnz, users, inter

    for _ in range(max(1, args.warmup)):
        with pkg.CooccurrenceCore(n_items=M, topk=topk, window_size_ms=1000, device=0) as warm:
            stream(warm, False)
    core = pkg.CooccurrenceCore(n_items=M, topk=topk, window_size_ms=1000, device=0)
    core.set_kernel_timing(True)
    lat, kms, pairs, nnz, users, inter = stream(core, True)
    total_pairs = int(np.sum(pairs))
    assert total_pairs == datagen.ordered_pairs(d["user_ptr"]), "the windows' pairs must add up to the whole log's"
    lat_ms = np.array(lat) * 1e3
    elapsed = float(np.sum(lat))
    # the counting kernel per window (HIP events on its stream): window pairs / expansion against resident histories
    b_alg = sum(algorithmic_bytes(p, n, u, k) for p, n, u, k in zip(pairs, inter, users, nnz))
    k_total = float(np.sum(kms)) * 1e-3
    achieved = b_alg / k_total / 1e9 if k_total > 0 else None
    out = {
        "metric": METRIC,
        "value": total_pairs / elapsed,
        "unit": "pairs/s",
        "n_gpus": 1,
        "steps": n_windows,
        "warmup": max(1, args.warmup),
        "ms_per_step": elapsed / n_windows * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {
            "workload": ("C4 (BASELINE configs[3]): the MovieLens-20M-shaped log (138,493 users x 26,744 items, 20,000,263 "
                         "interactions, datagen.config_c4 seed 4) over 100 tumbling 1 s windows into resident device state "
                         f"(histories, dense global rows, row sums), LLR top-{topk} of every touched row per window; a step "
                         "is one window (submit + finish, synchronised), value = the windows' incremental ordered pairs / "
                         "their summed latency"),
            "items": M, "windows": n_windows, "topk": topk, "ordered_pairs_total": total_pairs,
            "window_latency_ms": {"median": float(np.median(lat_ms)), "p90": float(np.percentile(lat_ms, 90)),
                                  "max": float(lat_ms.max()), "first": float(lat_ms[0])},
            "interactions_per_window_median": float(np.median(inter)),
        },
        "roofline": {
            "bound": "hbm", "kernel": "k_acc_batch (each window's expansion against the resident histories)",
            "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS if achieved else None, "traffic": None,
            "kernel_ms_total": k_total * 1e3, "algorithmic_bytes_total": b_alg,
            "note": "B_alg = sum over windows of 4P_w + 4N_w + 8(U_w+1) + 12D_w (the window's new pairs, new interactions, "
                    "active users, delta keys), over the summed HIP-event time of the counting kernel; the window latency "
                    "also holds the merge into the resident rows, the rescoring and the host bookkeeping (value)",
        },
        "cpu_baseline": None,
    }
    print(json.dumps(out), flush=True)
    core.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=["c3", "c5", "c2", "c4"], default="c3")
    ap.add_argument("--topk", type=int, default=50)
    ap.add_argument("--c5-part", type=int, default=0, help="C5 at N=1: the rank of the 8-GPU job whose unit is timed")
    ap.add_argument("--c5-world", type=int, default=8, help="C5 at N=1: the job's GPU count (owner map)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (default: the box's CPU share, OMP_NUM_THREADS, else every CPU)")
    ap.add_argument("--permute-items", action="store_true",
                    help="C3/C5: item ids through the fixed bijection datagen.c3_item_perm (ids not in popularity order)")
    ap.add_argument("--no-permuted", action="store_true",
                    help="C3 at N=1: skip the line's `permuted` sub-record (the same log with permuted item ids)")
    ap.add_argument("--ordered-rows", action="store_true",
                    help="C3: rows in column order (without it the counting line runs with COOC_FLAG_ANY_ORDER: a "
                         "row's entries in no particular order, as the reference's Int2ShortOpenHashMap rows)")
    args = ap.parse_args()
    if args.config == "c4":
        return run_c4(args)

    import torch
    import torch.distributed as dist

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen, sharding

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    large = args.config in ("c3", "c5")
    owner_unit = args.config == "c5" and world == 1
    if owner_unit:
        # C5 at N = 1: rank c5_part's unit of the c5_world-GPU job (module docstring)
        up, it = datagen.c3_log_device(dev, u1=args.c5_world * (datagen.C3_USERS // 8), permute=args.permute_items)
        M = datagen.C3_ITEMS
        tmp_core = pkg.CooccurrenceCore(n_items=M, device=local_rank)
        freq = tmp_core.item_counts(it)
        tmp_core.close()
        owner = sharding.snake_owner(freq, args.c5_world)
        rs_global = datagen.closed_form_rowsums_device(up, it, M)
        P_local = int(rs_global[owner == args.c5_part].sum().item())  # the owned rows' pairs (row sum = row's pairs)
        u0, u1 = 0, int(up.numel()) - 1
        kernel = "k_sp_main+k_sp_small+k_sp_tiny+k_sp_split_finalize"
        pmc = load_pmc(os.path.join(ROOT, "profiles", "pmc_k_sp_main.json"))
        workload = (f"C5 (BASELINE configs[4]) per-GPU unit of the {args.c5_world}-GPU job: the whole Zipf-skewed "
                    f"1B log resident (datagen.c3_users seed {datagen.C3_SEED}, {args.c5_world} x 1.25e6 users, 1e6 "
                    f"items, Zipf(1.0) with replacement, lognormal lengths of mean 100, one window; the state after "
                    f"the histories' all-gather), the rows rank {args.c5_part} owns (snake_owner of the whole log's "
                    f"item frequencies) counted over every user, each owned row scored by LLR against the whole "
                    f"log's row sums and observed total (the all-reduced row sums) with its top-{args.topk} kept "
                    f"(ItemRowRescorer...java:195-241)")
        if args.permute_items:
            workload += f"; item ids permuted by datagen.c3_item_perm (PCG64 seed {datagen.C3_PERM_SEED:#x})"
    elif large:
        U8 = datagen.C3_USERS // 8
        # the job's users [0, N U/8): contiguous ranges balanced on sum n_u (n_u - 1)
        lens_all = datagen.c3_lengths(0, world * U8)
        u0, u1 = sharding.balanced_user_ranges(np.concatenate([[0], np.cumsum(lens_all)]), world)[rank]
        up, it = datagen.c3_users(u0, u1, device=dev, permute=args.permute_items)
        M = datagen.C3_ITEMS
        P_local = int(np.sum(lens_all[u0:u1] * (lens_all[u0:u1] - 1)))
        # the timed span (HIP events on the stream): every counting kernel of the step -- k_sp_main (hash / dense
        # chunks, split shares), k_sp_small and k_sp_tiny (radix- and bitonic-sorted rows), k_sp_split_finalize
        kernel = "k_sp_main+k_sp_small+k_sp_tiny+k_sp_split_finalize"
        pmc = load_pmc(os.path.join(ROOT, "profiles", "pmc_k_sp_main.json"))
        workload = ("C3 Zipf-skewed 1B log (BASELINE configs[2]), shard-invariant generator "
                    f"datagen.c3_users seed {datagen.C3_SEED}: users [r*1.25e6, (r+1)*1.25e6) on rank r "
                    f"(1/8 of 1e7 users per GPU; the whole 1e9-interaction log at 8 GPUs), 1e6 items, Zipf(1.0) "
                    "with replacement, lognormal lengths of mean 100, one window")
        if args.permute_items:
            workload += (f"; item ids permuted by the fixed bijection datagen.c3_item_perm (PCG64 seed "
                         f"{datagen.C3_PERM_SEED:#x}): ids carry no popularity order")
        if args.config == "c5":
            workload = (f"C5 (BASELINE configs[4]): co-occurrence counts + LLR scoring of every entry + per-item "
                        f"top-{args.topk} (ItemRowRescorer...java:195-241) on " + workload[:1].lower() + workload[1:])
    else:
        d = datagen.config_c2(seed=2 + rank)
        up = torch.from_numpy(d["user_ptr"]).to(dev)
        it = torch.from_numpy(d["items"]).to(dev)
        M = d["n_items"]
        P_local = datagen.ordered_pairs(d["user_ptr"])
        kernel = "k_acc_batch"
        pmc = load_pmc(os.path.join(ROOT, "profiles", "pmc_k_acc_batch.json"))
        workload = ("C2 MovieLens-20M-shaped: 138,493 users x 26,744 items, 20,000,263 interactions per GPU, "
                    "Zipf(0.9) without replacement, one window, numpy PCG64 seed 2 (+rank)")
    U, N = int(up.numel()) - 1, int(it.numel())
    torch.cuda.synchronize()
    digest = source_digest()
    pmc_stale = bool(pmc) and pmc.get("source_digest") != digest
    if pmc_stale:  # counters of other code: not reported as this kernel's
        pmc = {"kernel": pmc.get("kernel"), "stale_source_digest": pmc.get("source_digest")}

    # C3 counts: the reference's rows are hash maps, so the count itself owes no column order (COOC_FLAG_ANY_ORDER;
    # consumers that want one pay for it: the host copies sort); C5 feeds the heaps in column order (the tie
    # contract of its parity tests)
    any_order = args.config == "c3" and not args.ordered_rows
    core = pkg.CooccurrenceCore(n_items=M, device=local_rank, any_order=any_order)
    core.set_kernel_timing(True)
    # N > 1, C3/C5: the exchange runs inside the library (cooc_count_owned / cooc_topk_owned) over its own RCCL
    # communicator; COOC_BENCH_EXCHANGE=torch keeps the torch.distributed orchestration of sharding.py
    lib_exchange = world > 1 and large and os.environ.get("COOC_BENCH_EXCHANGE", "library") != "torch"
    if lib_exchange:
        sharding.init_comm(core)

    topk_ms = []
    if args.config == "c5":
        tk_sizes = torch.empty(M, dtype=torch.int32, device=dev)
        tk_vals = torch.empty((M, args.topk), dtype=torch.int32, device=dev)
        tk_scores = torch.empty((M, args.topk), dtype=torch.float64, device=dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def count():
        if owner_unit:
            return core.count_device_owned(up, it, owner, args.c5_part, freq, N)
        if world == 1:
            return core.count_device(up, it)  # on torch's current stream; returns after it drained
        if large:
            return sharding.count_owned(core, up, it)
        return sharding.count_records(core, up, it)

    def step():
        r = count()
        if args.config == "c5":  # LLR + top-k of every (owned) row, resident on the device
            ev0.record()
            if owner_unit:
                core.topk_batch_device(args.topk, tk_sizes, tk_vals, tk_scores, rowsum_global=rs_global)
            elif world == 1:
                core.topk_batch_device(args.topk, tk_sizes, tk_vals, tk_scores)
            else:
                sharding.topk_owned(core, r, args.topk)
            ev1.record()
            ev1.synchronize()
            topk_ms.append(ev0.elapsed_time(ev1))
        return r

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

    # exactness checks of the last step's result on the device (outside the timed region): the in-kernel
    # row-sum check already failed the step if any row's counts missed W_a - c_a; here the whole output
    # is re-read: sum of all counts == sum of the row sums == the ordered pairs of the generator's
    # lengths, every row's columns strictly ascending, no zero count (cooc_verify_batch)
    chk = None
    if world == 1 or large:  # (the C2 records exchange's owner result is checked inside cooc_shard_count)
        chk = core.verify_batch()
        P_res = res.observed if world == 1 else res.local_observed
        assert chk["rows_bad_sum"] == 0 and chk["rows_bad_entries"] == 0, f"verify_batch: {chk}"
        assert chk["sum_counts"] == chk["sum_rowsums"] == P_res, f"verify_batch: {chk}, pairs {P_res}"
    if world == 1:
        assert res.observed == P_local, "pair count mismatch"
        D, P_counted, N_seen, U_seen = int(res.nnz), int(res.observed), N, U
    elif large:
        D, P_counted, N_seen, U_seen = int(res.owned.nnz), int(res.local_observed), res.n_interactions_all, res.n_users_all
    else:
        D, P_counted, N_seen, U_seen = int(res.owned.nnz), int(res.owned.observed), N, U
    # the same workload with its item ids permuted (datagen.c3_item_perm: ids carry no popularity order, as real
    # ids -- MovieLens, hashed -- do not), timed the same way: the id-order independence of the counting path
    permuted = None
    if large and world == 1 and args.config == "c3" and not args.permute_items and not args.no_permuted:
        del up, it
        up_p, it_p = datagen.c3_users(u0, u1, device=dev, permute=True)
        core.count_device(up_p, it_p)  # warm-up (allocations)
        torch.cuda.synchronize()
        n_p, kms_p = max(3, min(args.steps, 5)), []
        tp = time.perf_counter()
        for _ in range(n_p):
            r_p = core.count_device(up_p, it_p)
            kms_p.append(core.last_kernel_ms())
        torch.cuda.synchronize()
        el_p = time.perf_counter() - tp
        assert r_p.observed == P_local and int(r_p.nnz) == D, "permuted ids: a different result size"
        k_p = float(np.median(kms_p))
        permuted = {"workload": "the same users with item ids through datagen.c3_item_perm (PCG64 seed "
                                f"{datagen.C3_PERM_SEED:#x})", "steps": n_p, "ms_per_step": el_p / n_p * 1e3,
                    "value": P_local * n_p / el_p, "kernel_ms": k_p,
                    "frac": algorithmic_bytes(P_local, N, U, D) / (k_p * 1e-3) / 1e9 / HBM_PEAK_GBPS}
        del up_p, it_p
    stats = torch.tensor([elapsed, float(P_local), float(D)], dtype=torch.float64, device=dev)
    if world > 1:
        t = stats[:1].clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        s = stats[1:].clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        elapsed, p_total, d_total = float(t.item()), float(s[0].item()), float(s[1].item())
        if large:
            assert int(round(p_total)) == res.observed, "global pair count mismatch"
    else:
        p_total, d_total = float(P_local), float(D)
    ms_per_step = elapsed / args.steps * 1e3
    value = p_total * args.steps / elapsed

    k_ms = float(np.median(kernel_ms))
    b_alg = algorithmic_bytes(P_counted, N_seen, U_seen, D)
    achieved = b_alg / (k_ms * 1e-3) / 1e9
    traffic = pmc.get("hbm_bytes_per_launch")
    out = {
        "metric": METRIC,
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
            "workload": workload,
            "users_per_gpu": U, "items": M, "interactions_per_gpu": N, "ordered_pairs_total": int(p_total),
            "distinct_keys_total": int(d_total),
            "output": "padded CSR (row_base, row_nnz, col int32, cnt uint32) in HBM, exact counts" + (
                "; a row's entries in no particular order (COOC_FLAG_ANY_ORDER: hash chunks in slot order, as the "
                "reference's Int2ShortOpenHashMap rows)" if any_order else "; rows in column order"),
            "parallelism": f"users sharded over {world} GPU(s)" + (
                "; rows owned by frequency-snake order, histories all-gathered over RCCL" + (
                    " inside the library (cooc_count_owned)" if lib_exchange else " (torch.distributed)")
                if world > 1 and large else "; rows owned by a mod N, records exchange over RCCL" if world > 1 else ""),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kernel,
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            "traffic_kernels": (pmc.get("kernels") or pmc.get("kernel")) if traffic else None,
            "traffic_gbps": (traffic / (k_ms * 1e-3) / 1e9) if traffic else None,
            "hbm_frac_measured": (traffic / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS) if traffic else None,
            "lds_util": pmc.get("lds_util"),
            "lds_bank_conflict_frac": pmc.get("lds_bank_conflict_frac"),
            "l2_hit_rate": pmc.get("l2_hit_rate"),
            "wave_wait_frac": pmc.get("wave_wait_frac"),
            "limiter": limiter(pmc, traffic, k_ms),
            "pmc_source_digest": pmc.get("source_digest") or pmc.get("stale_source_digest"),
            "source_digest": digest,
            "pmc_stale": pmc_stale,
            "kernel_ms": k_ms,
            "algorithmic_bytes_per_launch": b_alg,
            "units_per_launch": {"ordered_pairs": P_counted, "interactions": N_seen, "users": U_seen,
                                 "distinct_keys": D},
            "note": "B_alg = 4P + 4N + 8(U+1) + 12D per launch of the dominant kernel (SURVEY.md §8(d); for C3 the "
                    "counting kernels together, which share the rows between them), divided by its time from HIP "
                    "events on its stream; frac > 1 would flag cache reuse. "
                    "traffic = HBM-side bytes per launch (C3: per step, summed over traffic_kernels, the same span) "
                    "from rocprofv3 PMC (2*FETCH_SIZE + WRITE_SIZE, profiles/pmc_<kernel>.json) when collected; see "
                    "DESIGN.md §4",
        },
        "cpu_baseline": None,
        "permuted": None,
        "checks": {"device_verify": chk, "in_kernel_row_sum_check": "every step (err bit -> exception)"},
    }
    if permuted is not None:
        permuted["vs_rank_ordered"] = permuted["ms_per_step"] / ms_per_step
        out["permuted"] = permuted
    if not large:
        # C2's dense-row kernel is bound by LDS atomics, not HBM (its HBM frac above 1 is the partner lists' reuse
        # from L2 / the Infinity Cache): one no-return ds_add_u32 per partner id a contribution walks -- sum_u n_u^2 =
        # P + N adds -- against the chip's measured random-slot rate (scripts/micro/lds_atomics.hip,
        # profiles/r02/micro/lds_atomics.txt: 6.89 lane-ops per CU-cycle, 4.23e12 adds/s at 2.4 GHz)
        adds = float(P_counted + N_seen)
        out["roofline_lds"] = {"bound": "lds_atomics", "kernel": "k_acc_batch", "achieved": adds / (k_ms * 1e-3),
                               "peak": LDS_ADD_PEAK, "unit": "ds_add lane-ops/s",
                               "frac": adds / (k_ms * 1e-3) / LDS_ADD_PEAK, "adds_per_launch": adds,
                               "lds_bank_conflict_frac": pmc.get("lds_bank_conflict_frac"),
                               "note": "sum_u n_u^2 no-return LDS adds per launch over the kernel's HIP-event time, against "
                                       "the random-slot ds_add rate measured on this chip (profiles/r02/micro)"}
    if args.config == "c5":
        out["config"]["topk"] = args.topk
        out["config"]["output"] += f"; top-{args.topk} heaps (sizes, values, scores) per row in HBM"
        out["topk_ms"] = tk = float(np.median(topk_ms))
        # the rescoring pass (cooc_topk_batch_device: k_col_terms + k_rescore) against its own bytes: every
        # entry streamed once (col + cnt, 8 B), the per-row CSR header and row sums (20 B per row), the heaps
        # written (sizes 4 B + k x (value 4 B + score 8 B) per row); the per-column LLR terms it gathers are
        # counted once (32 B per column) -- their re-reads hit L2 / the Infinity Cache
        pmc_rs = load_pmc(os.path.join(ROOT, "profiles", "pmc_k_rescore.json"))
        rs_stale = bool(pmc_rs) and pmc_rs.get("source_digest") != digest
        if rs_stale:
            pmc_rs = {"kernel": "k_rescore", "stale_source_digest": pmc_rs.get("source_digest")}
        # entries the kernel reads: a full heap whose root is NaN takes nothing more (score > NaN is false,
        # ItemRowRescorer...java:218-222), so k_rescore stops such a row after its first ceil(k / 64) * 64
        # entries; D_read counts what it does read (1 GPU: from the heaps and row lengths), not D
        d_read = entries_read(res, M, args.topk, tk_sizes, tk_scores) if world == 1 else None
        D_rs = d_read if d_read is not None else D
        # heaps whose root (the least score) is NaN: a wrapped int view makes a cell negative and its log NaN
        # (ItemRowRescorer...java:207-216 treats any NaN as fatal in DEVELOPMENT_MODE); nan_root_frac says how far
        # this unit is from that degenerate regime, entries_read / entries how much of the rows the kernel scored
        filled = tk_sizes > 0
        n_heaps = int(filled.sum().item())
        n_nan = int((filled & torch.isnan(tk_scores[:, 0])).sum().item())
        out["c5_regime"] = {"heaps": n_heaps, "nan_root_heaps": n_nan,
                            "nan_root_frac": n_nan / max(n_heaps, 1),
                            "entries_read_frac": (d_read / D) if (d_read is not None and D) else None,
                            "row_sums": "whole-log (closed form = the all-reduced owned row sums)" if owner_unit
                            else "this GPU's own result"}
        b_rs = 8.0 * D_rs + 20.0 * M + M * (4.0 + 12.0 * args.topk) + 32.0 * M
        a_rs = b_rs / (tk * 1e-3) / 1e9
        t_rs = pmc_rs.get("hbm_bytes_per_launch")
        # whole-log row sums (the owner unit): the two passes (cooc_stream.hip, k_rs_score then k_rs_heap) unless
        # COOC_RS_TWO_PASS=0; a GPU's own row sums: k_rescore3 (one pass; its rows end at a NaN heap root)
        tp_env = os.environ.get("COOC_RS_TWO_PASS")
        two_pass = (tp_env != "0") if owner_unit else (tp_env == "1")
        rs_kernel = ("k_col_terms+k_rs_tables+k_rs_bounds+k_rs_items+k_rs_score+k_rs_heap" if two_pass
                     else "k_col_terms+k_rescore3")
        out["roofline_rescore"] = {
            "bound": "hbm", "kernel": rs_kernel, "achieved": a_rs, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": a_rs / HBM_PEAK_GBPS, "traffic": t_rs, "kernel_ms": tk, "algorithmic_bytes_per_launch": b_rs,
            "units_per_launch": {"entries": D, "entries_read": d_read, "rows": M, "topk": args.topk},
            "traffic_gbps": (t_rs / (tk * 1e-3) / 1e9) if t_rs else None,
            "l2_hit_rate": pmc_rs.get("l2_hit_rate"), "wave_wait_frac": pmc_rs.get("wave_wait_frac"),
            "valu_busy": pmc_rs.get("valu_busy"), "limiter": limiter(pmc_rs, t_rs, tk),
            "pmc_source_digest": pmc_rs.get("source_digest") or pmc_rs.get("stale_source_digest"),
            "pmc_stale": rs_stale,
            # what the two passes move by design: pass 1 reads every entry (8 B) and writes its score's f32 bound
            # (4 B), pass 2 reads the bounds (4 B) of the entries it walks (rows end at a NaN root); the ~1% it
            # rescores exactly are not counted
            "two_pass_bytes_model": (12.0 * D + 4.0 * D_rs + 20.0 * M + M * (4.0 + 12.0 * args.topk) + 32.0 * M)
            if two_pass else None,
            "note": "B = 8D_read + 20M + M(4 + 12k) + 32M per launch (entries read: rows behind a NaN heap root "
                    "end early; row headers and sums, heaps, 32-B column terms), over the HIP-event time of the "
                    "rescoring call; the PMC (traffic, L2 hit) "
                    "shows how far the column-term gathers (one cache line per missed sparse entry) inflate the "
                    "bytes actually fetched (DESIGN.md §4)",
        }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if large:
            bu, bi = datagen.c3_users(0, 200_000, permute=args.permute_items)
            out["cpu_baseline"] = cpu_baseline(bu, bi, M, "the same C3 log", threads_override=args.cpu_threads)
        else:
            out["cpu_baseline"] = cpu_baseline(d["user_ptr"], d["items"], M, "the same C2 log",
                                               threads_override=args.cpu_threads)
    if rank == 0:
        print(json.dumps(out), flush=True)
    core.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
