#!/usr/bin/env python3
"""C5 stage at C2 scale: co-occurrence counts + LLR scoring of every row entry + per-item top-k
(k = 50 by default), one window over the C2-shaped log on one MI355X.

Times cooc_count_device and cooc_topk_batch separately (host wall around each, both synchronise).
Parity of the same computation is tests/test_gpu_parity.py::test_c2_scale_topk_rows.
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
    ap.add_argument("--topk", type=int, default=50)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen

    d = datagen.config_c2()
    up_h, it_h, M = d["user_ptr"], d["items"], d["n_items"]
    dev = torch.device("cuda", 0)
    up, it = torch.from_numpy(up_h).to(dev), torch.from_numpy(it_h).to(dev)
    core = pkg.CooccurrenceCore(n_items=M, device=0)
    res = core.count_device(up, it)
    core.topk_batch(args.topk)  # warm-up
    t_count, t_topk = [], []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = core.count_device(up, it)
        t1 = time.perf_counter()
        sizes, vals, scores = core.topk_batch(args.topk)
        t2 = time.perf_counter()
        t_count.append(t1 - t0)
        t_topk.append(t2 - t1)
    assert np.all(sizes <= args.topk)
    entries = int(res.nnz)
    out = {
        "config": f"C5 stage at C2 scale: LLR top-{args.topk} of all {M} rows after one window (C2 log, seed 2)",
        "count_ms": float(np.median(t_count) * 1e3),
        "topk_ms": float(np.median(t_topk) * 1e3),
        "entries_scored": entries,
        "llr_entries_per_s": entries / float(np.median(t_topk)),
        "topk_includes_copy_to_host": True,
    }
    print(json.dumps(out), flush=True)
    core.close()


if __name__ == "__main__":
    main()
