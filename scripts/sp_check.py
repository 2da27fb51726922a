#!/usr/bin/env python3
"""Debug harness for the large-universe path: counts users [0, 1e7 / shards) of the C3 log on the GPU
and checks a sample of rows for strictly ascending keys (a row whose tail was never written shows
trailing zeros).  Prints the failing rows with their contribution counts."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def d2h(ptr, n, dtype, offset=0):
    out = np.zeros(n, dtype)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr + offset * out.itemsize),
                             ctypes.c_size_t(out.nbytes), ctypes.c_int(2)) == 0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=64)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--rows", type=int, default=3000)
    args = ap.parse_args()
    import torch

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    if args.lib:
        sys.modules["flink_cooccurrence_amd._lib"].LIB_PATH = os.path.abspath(args.lib)
    from flink_cooccurrence_amd import datagen

    dev = torch.device("cuda", 0)
    U = datagen.C3_USERS // args.shards
    M = datagen.C3_ITEMS
    up, it = datagen.c3_users(0, U, device=dev)
    c = torch.bincount(it.long(), minlength=M).cpu().numpy()
    core = pkg.CooccurrenceCore(n_items=M, device=0)
    res = core.count_device(up, it)
    torch.cuda.synchronize()
    base = d2h(res.row_base, M, np.int64)
    nnz = d2h(res.row_nnz, M, np.int32)
    print("nnz", res.nnz, "sum row_nnz", int(nnz.sum()), flush=True)
    nzr = np.nonzero(nnz)[0]
    order = nzr[np.argsort(base[nzr], kind="stable")]
    ends = base[order] + nnz[order]
    ov = np.nonzero(base[order][1:] < ends[:-1])[0]
    print("rows with entries", len(nzr), "overlapping row regions", len(ov), flush=True)
    for k in ov[:10]:
        print("  overlap: row %d [%d, %d) and row %d [%d, %d)" % (order[k], base[order[k]], ends[k], order[k + 1],
                                                                base[order[k + 1]], ends[k + 1]), flush=True)
    rng = np.random.default_rng(1)
    sample = np.unique(np.concatenate([np.arange(0, 200), rng.integers(0, M, args.rows)]))
    bad = []
    for a in sample:
        cols = d2h(res.col, int(nnz[a]), np.int32, int(base[a]))
        if len(cols) > 1 and not np.all(np.diff(cols) > 0):
            k = int(np.argmax(np.diff(cols) <= 0))
            bad.append((int(a), int(c[a]), int(nnz[a]), k, int(cols[k]), int(cols[k + 1]), int(base[a])))
            if len(bad) <= 3:
                cnt = d2h(res.cnt, int(nnz[a]), np.uint32, int(base[a]))
                z = np.nonzero(cols[k + 1:] == 0)[0]
                nzt = np.nonzero(cols[k + 1:] != 0)[0]
                print("  row %d: zero cols after first-bad %d, nonzero after %d (first at +%s, last col %d), "
                      "cnt zeros in gap %d" % (a, len(z), len(nzt), nzt[0] if len(nzt) else "-", int(cols[-1]),
                                               int((cnt[k + 1:][cols[k + 1:] == 0] == 0).sum())), flush=True)
                if len(nzt):
                    j = k + 1 + nzt[0]
                    print("  resumes at", j, "cols", cols[j:j + 4].tolist(), "gap", j - k - 1, flush=True)
    print("checked", len(sample), "bad", len(bad), flush=True)
    for b in bad[:40]:
        print("row %d contribs %d nnz %d first-bad %d (%d -> %d) base %d" % b, flush=True)
    core.close()


if __name__ == "__main__":
    main()
