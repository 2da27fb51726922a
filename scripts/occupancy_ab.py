#!/usr/bin/env python3
"""Experiment: k_acc_batch time vs. workgroups per CU on a C2-shaped log folded to M items
(items mod M), so that the LDS row allows several workgroups per CU.  Occupancy is limited with
COOC_ACC_LDS_MIN (dynamic LDS inflated) and the grid with COOC_ACC_WGS."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen

    M = int(sys.argv[1]) if len(sys.argv) > 1 else 13372
    d = datagen.config_c2(seed=2)
    up_h, it_h = d["user_ptr"], (d["items"] % M).astype(np.int32)
    dev = torch.device("cuda", 0)
    up, it = torch.from_numpy(up_h).to(dev), torch.from_numpy(it_h).to(dev)
    core = pkg.CooccurrenceCore(n_items=M, device=0)
    core.set_kernel_timing(True)
    for _ in range(2):
        core.count_device(up, it)
    torch.cuda.synchronize()
    import time
    ks, t0 = [], time.perf_counter()
    for _ in range(8):
        core.count_device(up, it)
        ks.append(core.last_kernel_ms())
    dt = (time.perf_counter() - t0) / 8 * 1e3
    tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("COOC_"))
    print(f"M={M} {tag}: kernel {np.mean(ks):.3f} ms, step {dt:.3f} ms")
    core.close()


if __name__ == "__main__":
    main()
