"""Streaming windows across GPUs: p = 2 subtasks of the operator (NonSampledUserInteractionCounter...Operator
with the rows / row-sum windows and the rescorer, FlinkCooccurrences.java:65-74,135-167), each holding a
keyBy(user) shard of the records (:70) and its users' resident histories.  Every window, each subtask expands its
own users (NonSampled...java:129-161), and the library routes the partial delta rows to their owners (row a on
subtask a mod p: the keyBy(ItemCooccurrences::getItem) of :152), all-reduces the row-sum deltas (the broadcast
row-sum stream of :163) and the window's pairs; the owner merges its rows into its resident global rows and
rescores them (ItemRowRescorer...java:144-228).  The subtasks agree on every window they fire (the earliest due
on any of them, by an all-gather), so a subtask with no record in a window still joins its exchange.

Two processes on the box's one GPU, the communicator over gloo (cooc_comm_ops; RCCL refuses two ranks on one
GPU), 20+ windows of a C1-shaped click log, of a C4-shaped log (C2 lengths and popularity, without
replacement) and of a C1-shaped log over a 1e6-item universe (sparse resident rows; the owners merge
the partial rows by sorting), with the same or with different watermark sequences on the two subtasks: the union of the two subtasks' outputs equals OracleStream's, window by window (delta rows exact
and int16, row sums exact and int32, observed, top-k heaps), and the accumulators add up.  Needs an MI355X.
"""
import os
import pickle
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INT64_MAX = (1 << 63) - 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _records(kind):
    sys.path.insert(0, ROOT)
    import __graft_entry__

    __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen

    if kind == "c1":
        d = datagen.config_c1(seed=1, U=2000, M=300, mean=20.0)
        M = 300
    elif kind == "wide":  # a large universe (1e6 items: sparse resident rows, owners merge partial rows by sorting)
        M = 1_000_000
        d = datagen.config_c1(seed=5, U=2000, M=M, mean=20.0)
    else:
        d = datagen.config_c4(seed=4, n_windows=20, U=3000, M=2000, N=60_000)
        M = 2000
    users, items, ts = datagen.to_records(d["user_ptr"], d["items"], d["ts"])
    return users, items, ts, M


CHUNK = 4000


def _worker(rank, world, port, out_dir, kind, topk, lag=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import sharding

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    users, items, ts, M = _records(kind)
    op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1, "SECONDS", n_items=M, top_k=topk)
    sharding.init_comm_torch_ops(op.core)
    got = []
    for j, lo in enumerate(range(0, len(users), CHUNK)):
        sl = slice(lo, lo + CHUNK)
        mine = users[sl] % world == rank  # keyBy(0)
        op.process_elements(users[sl][mine], items[sl][mine], ts[sl][mine])
        # lag: subtask 1 receives only every third watermark (Flink's per-subtask minimum over input channels
        # that arrive in their own order), so the two subtasks call process_watermark different numbers of times
        if not (lag and rank == 1 and j % 3 != 2):
            got += op.process_watermark(int(ts[sl][-1]) - 1)
    got += op.process_watermark(INT64_MAX)
    out = dict(windows=got, acc=op.accumulators(), rowsums=op.core.global_rowsums(),
               rows={a: op.core.global_row(a) for a in range(rank, M, world * 7)})
    op.close()
    with open(os.path.join(out_dir, f"rank{rank}.pkl"), "wb") as f:
        pickle.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


def _union(parts):
    """The subtasks' outputs of one window as one WindowOutput-shaped record (each row on its owner only)."""
    from flink_cooccurrence_amd.core import WindowResult

    ts = {p.ts for p in parts}
    assert len(ts) == 1, f"subtasks fired different windows: {ts}"
    rows, rp, cols, exact, v16 = [], [0], [], [], []
    per_row = {}
    for p in parts:
        for r, a in enumerate(p.rows.tolist()):
            assert a not in per_row, f"row {a} emitted by two subtasks"
            s, e = int(p.row_ptr[r]), int(p.row_ptr[r + 1])
            per_row[a] = (p.cols[s:e], p.exact[s:e], p.v16[s:e])
    for a in sorted(per_row):
        c, x, v = per_row[a]
        rows.append(a)
        cols.append(c)
        exact.append(x)
        v16.append(v)
        rp.append(rp[-1] + len(c))
    rs = sorted((int(a), int(x), int(v)) for p in parts for a, x, v in zip(p.rs_items, p.rs_exact, p.rs_v32))
    tk = sorted((int(a), i, j) for j, p in enumerate(parts) for i, a in enumerate(p.topk_rows.tolist()))
    k = max((p.topk_values.shape[1] for p in parts if p.topk_values.ndim == 2), default=0)
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
    return WindowResult(
        ts=parts[0].ts, rows=np.array(rows, np.int32), row_ptr=np.array(rp, np.int64), cols=cat(cols, np.int32),
        exact=cat(exact, np.int64), v16=cat(v16, np.int16), rs_items=np.array([x[0] for x in rs], np.int32),
        rs_exact=np.array([x[1] for x in rs], np.int64), rs_v32=np.array([x[2] for x in rs], np.int32),
        observed=sum(int(p.observed) for p in parts), topk_rows=np.array([x[0] for x in tk], np.int32),
        topk_sizes=np.array([parts[j].topk_sizes[i] for _, i, j in tk], np.int32),
        topk_values=np.array([parts[j].topk_values[i] for _, i, j in tk], np.int32).reshape(len(tk), k),
        topk_scores=np.array([parts[j].topk_scores[i] for _, i, j in tk], np.float64).reshape(len(tk), k))


@pytest.mark.parametrize("kind,lag", [("c1", False), ("c4", False), ("c1", True), ("wide", False), ("wide", True)])
def test_two_subtasks_stream_vs_oracle(pkg, oracle, torch_cuda, tmp_path, kind, lag):
    """lag: the subtasks receive different watermark sequences; the windows still fire together, in order."""
    import torch.multiprocessing as mp

    from tests._helpers import assert_windows_equal

    world, topk = 2, 10
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), kind, topk, lag), nprocs=world, join=True)
    parts = [pickle.load(open(tmp_path / f"rank{r}.pkl", "rb")) for r in range(world)]
    users, items, ts, M = _records(kind)
    ref = oracle.OracleStream(1000, topk=topk)
    want = []
    for lo in range(0, len(users), CHUNK):
        sl = slice(lo, lo + CHUNK)
        ref.process_elements(users[sl], items[sl], ts[sl])
        want += ref.process_watermark(int(ts[sl][-1]) - 1)
    want += ref.process_watermark(INT64_MAX)
    n = [len(p["windows"]) for p in parts]
    assert n[0] == n[1] == len(want) >= 20, (n, len(want))
    for i, w in enumerate(want):
        assert_windows_equal(_union([p["windows"][i] for p in parts]), w)
    # accumulators: each subtask counts its own records / users' pairs / owned rows; the job's are the sums
    want_acc = ref.counters()
    acc = {k: sum(p["acc"][k] for p in parts) for k in parts[0]["acc"] if k != "rescorer_observed"}
    assert acc == {k: v for k, v in want_acc.items() if k != "rescorer_observed"}
    # (the rescorer's observed total is the job's on every subtask: it scores against the broadcast row sums)
    assert all(p["acc"]["rescorer_observed"] == want_acc["rescorer_observed"] for p in parts)
    # the resident state: every subtask holds the job's row sums, each row on its owner
    gi, gv32, gex = ref.global_rowsums()
    for p in parts:
        ex, v32 = p["rowsums"]
        assert np.array_equal(ex[gi], gex) and np.array_equal(v32[gi], gv32)
    rows, rp, cols, exact, v16 = ref.global_rows()
    pos = {int(a): r for r, a in enumerate(rows)}
    for p in parts:
        for a, (c, x, x16) in p["rows"].items():
            r = pos.get(a)
            if r is None:
                assert len(c) == 0
                continue
            assert np.array_equal(c, cols[rp[r]:rp[r + 1]]) and np.array_equal(x.astype(np.int64), exact[rp[r]:rp[r + 1]])


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch
