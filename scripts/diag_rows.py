#!/usr/bin/env python3
"""Diagnose rows of a C3-share result whose counts do not add up to their row sum: counts the bad
rows of a random sample through plain device-to-host copies (independent of cooc_verify_batch), and
shows where in the output region they sit."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def d2h(ptr, n, dtype, offset=0):
    out = np.zeros(n, dtype)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        src = ctypes.c_void_p(ptr + offset * out.itemsize)
        assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), src, ctypes.c_size_t(out.nbytes), ctypes.c_int(2)) == 0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--sample", type=int, default=3000)
    ap.add_argument("--lib", default=None, help="another build of libcooc_hip.so (e.g. an older one)")
    args = ap.parse_args()
    import torch

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    if args.lib:  # before the first call loads the library
        sys.modules["flink_cooccurrence_amd._lib"].LIB_PATH = os.path.abspath(args.lib)
        sys.modules["flink_cooccurrence_amd._lib"]._SIGS.pop("cooc_verify_batch", None)
        sys.modules["flink_cooccurrence_amd._lib"]._SIGS.pop("cooc_copy_window_delta_range", None)
    from flink_cooccurrence_amd import datagen

    dev = torch.device("cuda", 0)
    U, M = datagen.C3_USERS // args.shards, datagen.C3_ITEMS
    up, it = datagen.c3_users(0, U, device=dev)
    core = pkg.CooccurrenceCore(n_items=M, device=0)
    res = core.count_device(up, it)
    chk = core.verify_batch() if not args.lib else None
    base = d2h(res.row_base, M, np.int64)
    nnz = d2h(res.row_nnz, M, np.int32)
    rs = d2h(res.rowsum, M, np.int64)
    rng = np.random.default_rng(1)
    rows = np.flatnonzero(nnz > 0)
    sample = np.sort(rng.choice(rows, min(args.sample, len(rows)), replace=False))
    bad, good = [], []
    for a in sample.tolist():
        c = d2h(res.cnt, int(nnz[a]), np.uint32, int(base[a])).astype(np.int64)
        (bad if int(c.sum()) != int(rs[a]) else good).append(a)
    bad, good = np.array(bad, np.int64), np.array(good, np.int64)
    end = base + nnz
    out = {"verify": chk, "nnz_total": int(res.nnz), "sample": len(sample), "bad": len(bad),
           "max_end": int(end.max()), "bad_base_min": int(base[bad].min()) if len(bad) else None,
           "bad_base_max": int(base[bad].max()) if len(bad) else None,
           "good_base_max": int(base[good].max()) if len(good) else None,
           "bad_frac_above_2^32": float(np.mean(base[bad] >= 2**32)) if len(bad) else None,
           "good_frac_above_2^32": float(np.mean(base[good] >= 2**32)) if len(good) else None,
           "bad_rows_head": bad[:20].tolist()}
    # overlapping row regions?
    order = np.argsort(base[rows], kind="stable")
    b, e = base[rows][order], end[rows][order]
    out["overlapping_rows"] = int(np.sum(b[1:] < e[:-1]))
    # the first bad rows against rows summed directly from the users' lists
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_sparse import _Brute

    brute = _Brute(up.cpu().numpy(), it.cpu().numpy(), M)
    det = []
    for a in bad[:6].tolist():
        gc = d2h(res.col, int(nnz[a]), np.int32, int(base[a]))
        gn = d2h(res.cnt, int(nnz[a]), np.uint32, int(base[a])).astype(np.int64)
        wc, wn = brute.row(a)
        n = min(len(gc), len(wc))
        diff = np.flatnonzero((gc[:n] != wc[:n]) | (gn[:n] != wn[:n]))
        i = int(diff[0]) if len(diff) else n
        det.append({"row": a, "got_nnz": len(gc), "want_nnz": len(wc), "first_diff": i, "n_diff": int(len(diff)),
                    "zeros": int(np.sum(gn == 0)), "got": [gc[i:i + 6].tolist(), gn[i:i + 6].tolist()],
                    "want": [wc[i:i + 6].tolist(), wn[i:i + 6].tolist()],
                    "base": int(base[a]), "got_sum": int(gn.sum()), "want_sum": int(wn.sum()),
                    "diff_runs": int(np.sum(np.diff(diff) > 1)) + 1 if len(diff) else 0,
                    "last_diff": int(diff[-1]) if len(diff) else None})
    out["details"] = det
    print(json.dumps(out), flush=True)
    core.close()


if __name__ == "__main__":
    main()
