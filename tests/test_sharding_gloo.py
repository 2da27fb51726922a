"""The multi-GPU exchange (sharding.count_sharded) over world_size-2 gloo on CPU.

The device core is replaced by a numpy test double with the same interface (local reduce by the
oracle's closed form, owner-major packing, owner-side merge), so this checks the orchestration:
splits, ordering, the row-sum all-reduce and the global pair count.  The real pack/merge kernels
are checked on the GPU in test_gpu_parity.py::test_partition_pack_merge_kernels.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class FakeCore:
    def __init__(self, n_items):
        self.n_items = n_items

    def count_device(self, user_ptr, items, stream=None):
        from oracle import oracle

        rp, cols, data, rowsums, observed = oracle.closed_form(user_ptr.numpy(), items.numpy(), self.n_items)
        self.rp, self.cols, self.data, self.rowsums = rp, cols, data, rowsums

        class R:
            pass

        r = R()
        r.observed = observed
        return r

    def copy_rowsum_device(self, out, stream=None):
        out.copy_(torch.from_numpy(self.rowsums))

    def _order(self, n):
        return [a for o in range(n) for a in range(o, self.n_items, n)]

    def partition_plan(self, n):
        nnz = np.diff(self.rp)
        return np.array([nnz[o::n].sum() for o in range(n)], np.int64)

    def partition_pack(self, n, row_nnz, entries, stream=None):
        nnz = np.diff(self.rp)
        order = self._order(n)
        row_nnz.copy_(torch.from_numpy(nnz[order].astype(np.int32)))
        packed = [(self.cols[self.rp[a]:self.rp[a + 1]].astype(np.int64) << 32) | self.data[self.rp[a]:self.rp[a + 1]]
                  for a in order]
        if entries.numel():
            entries.copy_(torch.from_numpy(np.concatenate(packed)))

    def merge_partitions(self, n, part, recv_nnz, recv_entries, rowsum_global=None, stream=None):
        M = self.n_items
        R = len(range(part, M, n))
        nnz = recv_nnz.numpy().reshape(n, R)
        ent = recv_entries.numpy()
        off = np.concatenate([[0], np.cumsum(nnz.ravel())])
        rows = {}
        for r in range(R):
            acc = np.zeros(M, np.int64)
            for s in range(n):
                e = ent[off[s * R + r]:off[s * R + r + 1]]
                np.add.at(acc, (e >> 32).astype(np.int64), e & 0xFFFFFFFF)
            a = part + r * n
            rows[a] = acc
            if rowsum_global is not None:
                assert acc.sum() == int(rowsum_global[a])
        return rows


def _worker(rank, world, port, up_all, it_all, M, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__

    __graft_entry__.load_package()
    from flink_cooccurrence_amd import sharding

    # users sharded: contiguous user ranges
    U = len(up_all) - 1
    lo, hi = rank * U // world, (rank + 1) * U // world
    up = up_all[lo:hi + 1] - up_all[lo]
    it = it_all[up_all[lo]:up_all[hi]]
    core = FakeCore(M)
    res = sharding.count_sharded(core, torch.from_numpy(up), torch.from_numpy(it))
    out_q.put((rank, {a: v.tolist() for a, v in res.merged.items()}, res.rowsum.numpy().tolist(), res.observed))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_count_sharded_gloo(oracle, pkg, world):
    rng = np.random.default_rng(3)
    U, M = 90, 23
    lens = rng.integers(1, 12, U)
    up = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    it = rng.integers(0, M, up[-1]).astype(np.int32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, up, it, M, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
    C = np.zeros((M, M), np.int64)
    for a in range(M):
        C[a, cols[rp[a]:rp[a + 1]]] = data[rp[a]:rp[a + 1]]
    seen = set()
    for rank, rows, rs, obs in outs:
        assert obs == observed
        assert np.array_equal(np.array(rs), rowsums)
        for a, v in rows.items():
            assert a % world == rank
            assert np.array_equal(np.array(v), C[a])
            seen.add(a)
    assert seen == set(range(M))
