"""The multi-GPU orchestration (sharding.py) with the REAL device core: world_size 2, one process per
rank, both ranks on the box's one MI355X, torch.distributed over gloo (RCCL refuses two ranks on one
GPU; the gloo backend moves the same CUDA tensors through host memory).  Every collective the driver's
N-GPU bench issues -- the item-frequency all-reduce, the history all-to-alls of count_owned, the row-sum
all-reduce of topk_owned, the all-to-alls of count_records -- runs here between real library kernels
on torch's current stream, in the order the bench issues them.

Checked against one process counting the whole log (itself checked against the oracle elsewhere):
* count_owned (C3 / C5 path, n_items = 1e6): every rank's owned rows equal the whole log's rows, the
  other rows are empty, the owned parts cover every row; topk_owned's heaps (scores against the
  all-reduced row sums) equal the whole log's heaps row by row;
* count_records (C2 path, n_items < 40,320): the owned rows (part + r * world) equal the whole log's.
The keyBy(user) / keyBy(getItem) / broadcast() exchange of FlinkCooccurrences.java:70,152,163.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _d2h(ptr, n, dtype, offset=0):
    import ctypes

    out = np.zeros(n, dtype)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        src = ctypes.c_void_p(ptr + offset * out.itemsize)
        assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), src, ctypes.c_size_t(out.nbytes), ctypes.c_int(2)) == 0
    return out


def _rows(res, R):
    """(row_ptr, cols, cnt, rowsum) of the first R rows of a device result, packed."""
    base = _d2h(res.row_base, R, np.int64)
    nnz = _d2h(res.row_nnz, R, np.int32).astype(np.int64)
    rowsum = _d2h(res.rowsum, R, np.int64)
    rp = np.concatenate([[0], np.cumsum(nnz)])
    cols = np.zeros(int(rp[-1]), np.int32)
    cnt = np.zeros(int(rp[-1]), np.uint32)
    if res.dense:  # (records exchange at C2 density: rows are dense [R x M] counters)
        raise AssertionError("expected a CSR result")
    for a in np.flatnonzero(nnz):
        cols[rp[a]:rp[a + 1]] = _d2h(res.col, int(nnz[a]), np.int32, int(base[a]))
        cnt[rp[a]:rp[a + 1]] = _d2h(res.cnt, int(nnz[a]), np.uint32, int(base[a]))
    return rp, cols, cnt, rowsum


def _c3_log(n_users):
    sys.path.insert(0, ROOT)
    import __graft_entry__

    __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen

    up, it = datagen.c3_users(0, n_users)
    return up, it, datagen.C3_ITEMS


def _c2_log():
    from flink_cooccurrence_amd import datagen

    up, it = datagen.small_log(seed=9, U=2000, M=3000, mean_len=25.0, replacement=False)
    return up, it, 3000


def _worker(rank, world, port, out_dir, n_users, topk, exchange):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import sharding

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    # ---- C3 / C5 path: histories all-gathered, owned rows counted, top-k against all-reduced row sums
    up, it, M = _c3_log(n_users)
    u0, u1 = sharding.balanced_user_ranges(up, world)[rank]
    lo, hi = int(up[u0]), int(up[u1])
    up_r = torch.from_numpy(up[u0:u1 + 1] - lo).to(dev)
    it_r = torch.from_numpy(it[lo:hi]).to(dev)
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        if exchange in ("library", "library_host"):  # cooc_count_owned(_host): the exchange inside the library
            sharding.init_comm_torch_ops(core)
        if exchange == "library_host":  # a JVM subtask's call: host arrays in, the owned rows copied out
            b, info = core.count_owned_host(up[u0:u1 + 1] - lo, it[lo:hi])
            out.update(c3_rp=b.row_ptr, c3_cols=b.cols, c3_cnt=b.cnt, c3_rowsum=b.rowsum,
                       c3_owner=_d2h(info.owner, M, np.int32), c3_observed=np.int64(info.observed),
                       c3_local_observed=np.int64(info.local_observed), c3_n_all=np.int64(info.n_interactions_all))
            res = sharding.OwnedResult(info.part, info.n_parts, None, None, int(info.observed),
                                       int(info.local_observed), int(info.n_users_all),
                                       int(info.n_interactions_all), int(info.gathered_bytes))
            res.owner = torch.from_numpy(out["c3_owner"]).to(dev)
        else:
            res = sharding.count_owned(core, up_r, it_r)
            torch.cuda.current_stream().synchronize()
            rp, cols, cnt, rowsum = _rows(res.owned, M)
            out.update(c3_rp=rp, c3_cols=cols, c3_cnt=cnt, c3_rowsum=rowsum, c3_owner=res.owner.cpu().numpy(),
                       c3_observed=np.int64(res.observed), c3_local_observed=np.int64(res.local_observed),
                       c3_n_all=np.int64(res.n_interactions_all))
        tk = sharding.topk_owned(core, res, topk)
        torch.cuda.current_stream().synchronize()
        out.update(tk_sizes=tk.sizes.cpu().numpy(), tk_values=tk.values.cpu().numpy(),
                   tk_scores=tk.scores.cpu().numpy(), tk_rowsum=tk.rowsum.cpu().numpy())
    # ---- C2 path (n_items < 40,320): records routed to owner(a) = a mod world
    up, it, M = _c2_log()
    u0, u1 = sharding.balanced_user_ranges(up, world)[rank]
    lo, hi = int(up[u0]), int(up[u1])
    with pkg.CooccurrenceCore(n_items=M, device=0, output="csr") as core:
        rr = sharding.count_records(core, torch.from_numpy(up[u0:u1 + 1] - lo).to(dev),
                                    torch.from_numpy(it[lo:hi]).to(dev))
        torch.cuda.current_stream().synchronize()
        R = sharding.rows_owned(M, world, rank)
        rp, cols, cnt, rowsum = _rows(rr.owned, R)
        out.update(c2_rp=rp, c2_cols=cols, c2_cnt=cnt, c2_rowsum=rowsum, c2_observed=np.int64(rr.observed))
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("exchange", ["torch", "library", "library_host"])
def test_two_ranks_real_core_vs_one_process(pkg, torch_cuda, tmp_path, exchange):
    """exchange "torch": sharding.py moves the buffers over torch.distributed; "library": the whole C3 step
    is cooc_count_owned / cooc_topk_owned, the library's exchange over cooc_comm_ops callbacks (gloo here,
    RCCL in production: the same orchestration code); "library_host": cooc_count_owned_host from host
    arrays and cooc_copy_batch of the owned rows, the calls a JVM subtask makes."""
    import torch
    import torch.multiprocessing as mp

    world, n_users, topk = 2, 4000, 10
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), n_users, topk, exchange), nprocs=world, join=True)
    parts = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]

    # the whole log in one process
    up, it, M = _c3_log(n_users)
    dev = torch.device("cuda")
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        whole = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
        torch.cuda.current_stream().synchronize()
        w_rp, w_cols, w_cnt, w_rowsum = _rows(whole, M)
        sizes = torch.empty(M, dtype=torch.int32, device=dev)
        vals = torch.empty((M, topk), dtype=torch.int32, device=dev)
        scores = torch.empty((M, topk), dtype=torch.float64, device=dev)
        core.topk_batch_device(topk, sizes, vals, scores)
        torch.cuda.current_stream().synchronize()
        w_sz, w_v, w_sc = sizes.cpu().numpy(), vals.cpu().numpy(), scores.cpu().numpy()
    lens = np.diff(up)
    P = int(np.sum(lens * (lens - 1)))
    owner = parts[0]["c3_owner"]
    assert np.array_equal(owner, parts[1]["c3_owner"]), "ranks computed different owner maps"
    covered = np.zeros(M, bool)
    w_nnz = np.diff(w_rp)
    for r, p in enumerate(parts):
        assert int(p["c3_observed"]) == P and int(p["c3_n_all"]) == len(it)
        nnz = np.diff(p["c3_rp"])
        mine = owner == r
        covered |= mine
        assert np.all(nnz[~mine] == 0)
        assert np.array_equal(nnz[mine], w_nnz[mine]) and np.array_equal(p["c3_rowsum"][mine], w_rowsum[mine])
        for a in np.flatnonzero(mine & (w_nnz > 0)):
            sl, ws = slice(p["c3_rp"][a], p["c3_rp"][a + 1]), slice(w_rp[a], w_rp[a + 1])
            # (device rows are in column order, cooc_copy_batch's in ascending ids: compared as sorted rows)
            o1, o2 = np.argsort(p["c3_cols"][sl], kind="stable"), np.argsort(w_cols[ws], kind="stable")
            assert np.array_equal(p["c3_cols"][sl][o1], w_cols[ws][o2]), f"row {a}"
            assert np.array_equal(p["c3_cnt"][sl][o1], w_cnt[ws][o2]), f"row {a}"
        # top-k: the all-reduced row sums are the whole log's, so the owned heaps are the whole log's heaps
        assert np.array_equal(p["tk_rowsum"], w_rowsum)
        sz = p["tk_sizes"]
        assert np.all(sz[~mine] == 0) and np.array_equal(sz[mine], w_sz[mine])
        for a in np.flatnonzero(mine & (w_sz > 0)):
            n = int(w_sz[a])
            assert np.array_equal(p["tk_values"][a, :n], w_v[a, :n]), f"row {a}"
            # (NaN scores exist: the reference's k22 = observed + k11 - k12 - k21 can go negative)
            assert np.array_equal(p["tk_scores"][a, :n], w_sc[a, :n], equal_nan=True), f"row {a}"
    assert covered.all()
    assert sum(int(p["c3_local_observed"]) for p in parts) == P

    # C2 records exchange: owned rows part + r * world of the whole log
    up, it, M = _c2_log()
    with pkg.CooccurrenceCore(n_items=M, device=0, output="csr") as core:
        whole = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
        torch.cuda.current_stream().synchronize()
        w_rp, w_cols, w_cnt, w_rowsum = _rows(whole, M)
    lens = np.diff(up)
    for r, p in enumerate(parts):
        assert int(p["c2_observed"]) == int(np.sum(lens * (lens - 1)))
        for i, a in enumerate(range(r, M, world)):
            sl, ws = slice(p["c2_rp"][i], p["c2_rp"][i + 1]), slice(w_rp[a], w_rp[a + 1])
            assert np.array_equal(p["c2_cols"][sl], w_cols[ws]) and np.array_equal(p["c2_cnt"][sl], w_cnt[ws]), f"row {a}"
            assert p["c2_rowsum"][i] == w_rowsum[a]


def test_rccl_world1_count_owned_equals_count_device(pkg, torch_cuda):
    """The RCCL transport (cooc_comm_init over librccl.so.1) at world size 1: cooc_count_owned (item counts
    all-reduced, owner map, history exchange, owned count, pairs all-reduced -- every collective through
    RCCL) owns every row and equals cooc_count_device; cooc_topk_owned equals the batch top-k."""
    import torch

    up, it, M = _c3_log(3000)
    dev = torch.device("cuda", 0)
    up_d, it_d = torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev)
    topk = 10
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        whole = core.count_device(up_d, it_d)
        torch.cuda.current_stream().synchronize()
        w = _rows(whole, M)
        sizes = torch.empty(M, dtype=torch.int32, device=dev)
        vals = torch.empty((M, topk), dtype=torch.int32, device=dev)
        scores = torch.empty((M, topk), dtype=torch.float64, device=dev)
        core.topk_batch_device(topk, sizes, vals, scores)
        torch.cuda.current_stream().synchronize()
        w_tk = (sizes.cpu().numpy(), vals.cpu().numpy(), scores.cpu().numpy())
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        core.comm_init(core.comm_unique_id(), 0, 1)
        res, info = core.count_owned(up_d, it_d)
        torch.cuda.current_stream().synchronize()
        o = _rows(res, M)
        lens = np.diff(up)
        assert info.observed == info.local_observed == int(np.sum(lens * (lens - 1)))
        assert info.n_users_all == len(lens) and info.n_interactions_all == len(it) and info.gathered_bytes == 0
        assert np.all(_d2h(info.owner, M, np.int32) == 0)
        assert np.array_equal(_d2h(info.item_counts, M, np.int64), np.bincount(it, minlength=M))
        for x, y in zip(o, w):
            assert np.array_equal(x, y)
        rs = torch.empty(M, dtype=torch.int64, device=dev)
        core.topk_owned(topk, sizes, vals, scores, rowsum_global=rs)
        torch.cuda.current_stream().synchronize()
        assert np.array_equal(rs.cpu().numpy(), w[3])
        assert np.array_equal(sizes.cpu().numpy(), w_tk[0]) and np.array_equal(vals.cpu().numpy(), w_tk[1])
        assert np.array_equal(scores.cpu().numpy(), w_tk[2], equal_nan=True)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch
