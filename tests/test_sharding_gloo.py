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


class FakeRecordsCore:
    """numpy double of the sharded-records entry points, restating their buffer contract
    (include/cooc.h: cooc_shard_plan / cooc_shard_count): padded u16 arena with sink id M, 8-B
    descriptors (n_u << 40 | arena offset) grouped by owner then owned row, owner-major row counts."""

    def __init__(self, n_items):
        self.n_items = n_items

    @staticmethod
    def shard_arena_cap(n_users, n):
        return (n + 7 * max(n_users, 1) + 16 + 7) // 8 * 8

    def shard_plan(self, user_ptr, items, W, desc, row_counts, arena, stream=None):
        M = self.n_items
        up, it = user_ptr.numpy(), items.numpy()
        lens = np.diff(up)
        plen = (lens + 7) // 8 * 8
        poff = np.concatenate([[0], np.cumsum(plen)])
        ar = np.full(len(arena), M, np.int64)
        for j in range(len(lens)):
            ar[poff[j]:poff[j] + lens[j]] = it[up[j]:up[j + 1]]
        arena.copy_(torch.from_numpy(ar.astype(np.uint16).view(np.int16)))
        users = np.repeat(np.arange(len(lens)), lens)
        owner_rows = [list(range(o, M, W)) for o in range(W)]
        order = [a for rows in owner_rows for a in rows]
        d, rc = [], []
        for a in order:
            js = users[it == a]
            rc.append(len(js))
            d.extend(int((lens[j] << 40) | poff[j]) for j in js)
        if len(d):
            desc.copy_(torch.tensor(d, dtype=torch.int64))
        row_counts.copy_(torch.tensor(rc, dtype=torch.int32))
        send = np.array([sum(rc[len(sum(owner_rows[:o], [])):len(sum(owner_rows[:o + 1], []))]) for o in range(W)],
                        np.int64)
        return send, int(poff[-1]), int(np.sum(lens * (lens - 1)))

    def shard_count(self, W, part, recv_rc, recv_desc, arena_all, stride, stream=None):
        M = self.n_items
        R = len(range(part, M, W))
        rc = recv_rc.numpy().reshape(W, R)
        d = recv_desc.numpy().astype(np.uint64)
        ar = arena_all.numpy().view(np.uint16).astype(np.int64)
        src = np.concatenate([[0], np.cumsum(rc.ravel())])
        rows = {}
        for r in range(R):
            acc = np.zeros(M + 1, np.int64)
            n_c = 0
            for s_ in range(W):
                for k in range(src[s_ * R + r], src[s_ * R + r + 1]):
                    l, off = int(d[k] >> np.uint64(40)), int(d[k] & np.uint64((1 << 40) - 1)) + s_ * stride
                    np.add.at(acc, ar[off:off + l], 1)
                    n_c += 1
            a = part + r * W
            acc[a] -= n_c
            rows[a] = acc[:M]
        return rows


class FakeOwnedCore:
    """numpy double of cooc_count_device_owned (include/cooc.h): the rows a with owner[a] == part of
    the closed form over every user given; returns {row: dense counts} plus the owned rows' pairs."""

    def __init__(self, n_items):
        self.n_items = n_items

    def item_counts(self, items, out=None, stream=None):
        return torch.from_numpy(np.bincount(items.numpy(), minlength=self.n_items).astype(np.int64))

    def count_device_owned(self, user_ptr, items, owner, part, item_counts, n_total, stream=None):
        from oracle import oracle

        M = self.n_items
        up, it = user_ptr.numpy(), items.numpy()
        assert int(item_counts.sum()) == n_total == len(it)
        assert np.array_equal(item_counts.numpy(), np.bincount(it, minlength=M))
        rp, cols, data, rowsums, _ = oracle.closed_form(up, it, M)
        own = owner.numpy()

        class R:
            pass

        r = R()
        r.rows = {}
        for a in range(M):
            if own[a] == part:
                v = np.zeros(M, np.int64)
                v[cols[rp[a]:rp[a + 1]]] = data[rp[a]:rp[a + 1]]
                r.rows[a] = v
        r.observed = int(sum(rowsums[a] for a in r.rows))
        r.nnz = int(sum(np.count_nonzero(v) for v in r.rows.values()))
        self.rows = r.rows
        self.rowsum = np.where(own == part, rowsums, 0).astype(np.int64)
        return r

    def copy_rowsum_device(self, out, stream=None):
        out.copy_(torch.from_numpy(self.rowsum))

    def topk_batch_device(self, topk, sizes, values, scores, rowsum_global=None, exact_scores=False, stream=None):
        """cooc_topk_batch_device over the owned rows, scored with the given (all-reduced) row sums."""
        from oracle import oracle
        from tests._helpers import oracle_row_topk

        rs32 = rowsum_global.numpy().astype(np.int32).astype(np.int64)
        sizes.zero_()
        for a, v in self.rows.items():
            nz = np.flatnonzero(v)
            heap = oracle_row_topk(oracle, nz, v[nz].astype(np.int16), rs32, a, topk, int(rs32.sum()))
            sizes[a] = len(heap)
            for i, (b, sc) in enumerate(heap):
                values[a, i] = b
                scores[a, i] = sc


def _worker(rank, world, port, up_all, it_all, M, out_q, mode="partials"):
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
    if mode in ("owned", "owned_topk"):
        core = FakeOwnedCore(M)
        res = sharding.count_owned(core, torch.from_numpy(up), torch.from_numpy(it))
        rows, rs = res.owned.rows, None
        owner = res.owner.numpy()
        assert all(owner[a] == rank for a in rows)
        if mode == "owned_topk":  # C5: heaps of the owned rows against the all-reduced row sums
            tk = sharding.topk_owned(core, res, 5)
            rs = tk.rowsum.numpy().tolist()
            rows = {a: (int(tk.sizes[a]), tk.values[a].tolist(), tk.scores[a].tolist()) for a in rows}
            assert all(int(tk.sizes[a]) == 0 for a in range(M) if owner[a] != rank)
    elif mode == "records":
        res = sharding.count_records(FakeRecordsCore(M), torch.from_numpy(up), torch.from_numpy(it))
        rows, rs = res.owned, None
    else:
        res = sharding.count_sharded(FakeCore(M), torch.from_numpy(up), torch.from_numpy(it))
        rows, rs = res.merged, res.rowsum.numpy().tolist()
    out_q.put((rank, {a: (v.tolist() if hasattr(v, "tolist") else v) for a, v in rows.items()}, rs, res.observed))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_snake_owner_balances_zipf(pkg):
    """Rows by descending frequency dealt in snake order: Zipf-hot rows land on different ranks and the
    ranks' frequency mass is close to equal."""
    from flink_cooccurrence_amd import sharding

    counts = torch.tensor(np.round(1e7 / np.arange(1, 100_001)).astype(np.int64))
    for W in (2, 4, 8):
        own = sharding.snake_owner(counts, W).numpy()
        assert sorted(own[:W].tolist()) == list(range(W))
        mass = np.bincount(own, weights=counts.numpy(), minlength=W)
        assert mass.max() / mass.mean() < 1.03


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_library_snake_owner_equals_python(pkg, world):
    """cooc_snake_owner (the owner map cooc_count_owned builds inside the library) == sharding.snake_owner,
    ties in the frequencies included (a smaller id first; a smaller rank first at equal load)."""
    from flink_cooccurrence_amd import core, sharding

    rng = np.random.default_rng(world)
    for counts in (np.round(1e7 / np.arange(1, 60_001)).astype(np.int64), rng.integers(0, 50, 30_000),
                   np.zeros(100, np.int64), np.array([5], np.int64)):
        want = sharding.snake_owner(torch.from_numpy(counts), world).numpy()
        assert np.array_equal(core.CooccurrenceCore.snake_owner(counts, world), want)
        assert np.array_equal(core.CooccurrenceCore.snake_owner(counts, world, head=7),
                              sharding.snake_owner(torch.from_numpy(counts), world, head=7).numpy())


@pytest.mark.parametrize("world,mode", [(2, "partials"), (3, "partials"), (2, "records"), (3, "records"), (2, "owned"),
                                        (3, "owned"), (2, "owned_topk"), (3, "owned_topk")])
def test_count_sharded_gloo(oracle, pkg, world, mode):
    rng = np.random.default_rng(3)
    U, M = 90, 23
    lens = rng.integers(1, 12, U)
    up = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    it = rng.integers(0, M, up[-1]).astype(np.int32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, up, it, M, q, mode)) for r in range(world)]
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
    rs32 = rowsums.astype(np.int32).astype(np.int64)
    for rank, rows, rs, obs in outs:
        assert obs == observed
        if rs is not None:
            assert np.array_equal(np.array(rs), rowsums)
        for a, v in rows.items():
            if mode not in ("owned", "owned_topk"):
                assert a % world == rank
            if mode == "owned_topk":  # the whole log's heap of row a
                from tests._helpers import assert_row_topk, oracle_row_topk

                nz = np.flatnonzero(C[a])
                want = oracle_row_topk(oracle, nz, C[a][nz].astype(np.int16), rs32, a, 5, int(rs32.sum()))
                assert_row_topk(v[0], v[1], v[2], want, where=f"row {a}")
                seen.add(a)
                continue
            assert np.array_equal(np.array(v), C[a])
            assert a not in seen
            seen.add(a)
    assert seen == set(range(M))


def test_balanced_user_ranges(pkg):
    """Contiguous user ranges balanced on sum n_u (n_u - 1): they tile the users, and on a
    skewed log every rank's pair work is within one user's work of the mean."""
    from flink_cooccurrence_amd import datagen, sharding

    up, it = datagen.c3_users(0, 20_000)
    n = np.diff(up)
    w = n * (n - 1)
    for world in (1, 2, 3, 8):
        rng = sharding.balanced_user_ranges(up, world)
        assert rng[0][0] == 0 and rng[-1][1] == len(n)
        assert all(rng[r][1] == rng[r + 1][0] for r in range(world - 1))
        work = np.array([w[a:b].sum() for a, b in rng])
        assert work.sum() == w.sum()
        assert np.all(np.abs(work - w.sum() / world) <= w.max() + 1)
        sup, sit, u0 = sharding.shard_users(up, it, world, world - 1)
        assert u0 == rng[-1][0] and sup[0] == 0 and len(sit) == sup[-1] == up[rng[-1][1]] - up[rng[-1][0]]
    t = torch.from_numpy(up)
    assert sharding.balanced_user_ranges(t, 4) == sharding.balanced_user_ranges(up, 4)


def _gather_worker(rank, world, port, sizes, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__

    __graft_entry__.load_package()
    from flink_cooccurrence_amd import sharding

    part = torch.arange(sizes[rank], dtype=torch.int32) + 1000 * rank
    out = torch.full((sum(sizes),), -1, dtype=torch.int32)
    sharding._gather_parts(out, part, sizes)
    out_q.put((rank, out.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("sizes", [[5, 0, 7], [0, 3], [4, 4, 4, 0]])
def test_gather_parts_uneven_gloo(pkg, sizes):
    """count_owned's history all-gather (one uneven all_to_all_single per array): the ranks' parts land
    compact and in rank order on every rank, empty parts included."""
    world = len(sizes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [v for r in range(world) for v in range(1000 * r, 1000 * r + sizes[r])]
    for r in range(world):
        assert outs[r] == want
