"""The JNI call sequence of the p > 1 one-window Flink operators (GpuOwnedCooccurrenceRowsOperator and
GpuOwnedCooccurrenceTopKOperator, flink-cooccurrence_amd/jvm), replayed through the same C-ABI by two
processes -- one per Flink subtask -- whose communicator is the library's cooc_comm_ops transport over gloo
(RCCL refuses two ranks on one GPU).  What each subtask does, in the Java operators' order:

  processElement   buffer (user, item, ts) of its keyBy(user) shard;
  processWatermark at every watermark that passes a new window end, cooc_comm_allgather_i64 of the subtask's
                   window start (Long.MIN_VALUE: no records yet); the window whose end the watermark passed
                   fires on EVERY subtask (one with no records joins the same collective), two different
                   windows are an IllegalStateException;
  fire             the shard as CSR -> cooc_count_owned_host (item counts all-reduced, owner map, histories
                   exchanged, owned rows counted) -> rows operator: cooc_copy_batch row offsets, then the
                   entries in row ranges of at most MAX_RANGE_ENTRIES (forced small here: 5,000) with
                   cooc_copy_batch_range, one Int2ShortOpenHashMap per owned row plus its int row sum
                   (ItemRowAggregator.java:50-56, RowSumAggregator.java:66); top-k operator:
                   cooc_topk_owned_host -> cooc_copy_topk_batch_range in row ranges -> one
                   IntDoublePriorityQueue per owned row with entries (ItemRowRescorer...java:224-226).

Checked against the oracle on the whole log: the union of the subtasks' rows is the closed form's matrix in
the reference's int16 view, the row sums its int32 view, and every emitted heap the oracle's rescorer loop
(ItemRowRescorer...java:195-223, LogLikelihood.java:41-57, IntDoublePriorityQueue.java:132-205) fed the row
in the device's order, within SURVEY §8(a)'s tolerance.  Needs an MI355X.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LONG_MIN = -(1 << 63)
WINDOW_MS = 1000
MAX_RANGE_ENTRIES = 5000  # (CoocWindowReader / CoocBatchReader use 1 << 24; small here so ranges are many)
TOPK_ROWS_PER_RANGE = 4096


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _log(n_users):
    sys.path.insert(0, ROOT)
    import __graft_entry__

    __graft_entry__.load_package()
    from flink_cooccurrence_amd import datagen

    up, it = datagen.c3_users(0, n_users)
    return up, it, datagen.C3_ITEMS


def _records(up, it, seed=7):
    """The log as Tuple3(user, item, ts) records in one interleaved arrival order (per-user order kept),
    timestamps ascending inside window [5000, 6000)."""
    rng = np.random.default_rng(seed)
    users = np.repeat(np.arange(len(up) - 1), np.diff(up))
    seq = users[rng.permutation(len(it))]  # a random interleave of the users' occurrences
    # the j-th occurrence of user u in seq carries u's j-th item (up is the CSR of users in ascending order)
    idx = np.empty(len(it), np.int64)
    idx[np.argsort(seq, kind="stable")] = np.arange(len(it))
    ts = 5000 + (np.arange(len(it)) * 999) // max(len(it), 1)
    return seq.astype(np.int32), it[idx].astype(np.int32), ts.astype(np.int64)


class _OwnedSubtask:
    """The Java operators' state and calls (GpuOwnedCooccurrence{Rows,TopK}Operator, OwnedExchange) on one
    handle."""

    def __init__(self, core, n_items, topk):
        self.core, self.n_items, self.topk = core, n_items, topk
        self.users, self.items = [], []
        self.window_start = LONG_MIN
        self.watermark = LONG_MIN  # this subtask's own (timerService.currentWatermark())
        self.agreed = LONG_MIN     # the minimum watermark over the subtasks at the last agreement step
        self.fired = False
        self.late = 0              # UserInteractionCounterLateElements

    def process_element(self, user, item, ts):
        if ts <= self.watermark:  # NonSampled...java:89-91: dropped and counted
            self.late += 1
            return
        start = ts - ts % WINDOW_MS
        if self.window_start == LONG_MIN:
            self.window_start = start
        elif start != self.window_start or self.fired:
            raise RuntimeError(f"one window per operator; record at {ts}")
        self.users.append(user)
        self.items.append(item)

    def process_watermark(self, mark):
        """-> the fired window's outputs, or None.  Collective: runs agreement steps while this subtask's
        watermark is ahead of the agreed minimum (OwnedExchange.fireAt)."""
        self.watermark = max(self.watermark, mark)
        while not self.fired and self.watermark > self.agreed:
            wmin = min(int(w) for w in self.core.comm_allgather_i64(self.watermark))
            starts = self.core.comm_allgather_i64(self.window_start)
            known = sorted({int(s) for s in starts if s != LONG_MIN})
            if len(known) > 1:
                raise RuntimeError(f"subtasks hold records of different windows: {known}")
            self.agreed = max(self.agreed, wmin)
            if known and known[0] + WINDOW_MS - 1 <= self.agreed:
                self.fired = True
                return self._fire(known[0] + WINDOW_MS - 1)
        return None

    def _fire(self, timestamp):
        u = np.asarray(self.users, np.int64)
        it = np.asarray(self.items, np.int32)
        o = np.argsort(u, kind="stable")  # users ascending, each user's items in arrival order
        it = it[o]
        bounds = np.flatnonzero(np.diff(u[o])) + 1 if len(u) else np.zeros(0, np.int64)
        up = np.concatenate([[0], bounds, [len(u)]]).astype(np.int64) if len(u) else np.zeros(1, np.int64)
        winfo, info = self.core.count_owned_host_info(up, it)
        # rows operator: offsets once, then row ranges of at most MAX_RANGE_ENTRIES entries
        rp, _rs, rs32 = self.core.copy_batch_row_ptr()
        rows = {}
        M, r0 = self.n_items, 0
        n_ranges = 0
        while r0 < M:
            r1 = r0 + 1
            while r1 < M and rp[r1 + 1] - rp[r0] <= MAX_RANGE_ENTRIES:
                r1 += 1
            n = int(rp[r1] - rp[r0])
            cols, _cnt, cnt16 = self.core.copy_batch_range(r0, r1, max(n, 1))
            n_ranges += 1
            for a in range(r0, r1):
                f, t = int(rp[a] - rp[r0]), int(rp[a + 1] - rp[r0])
                if t > f:
                    rows[a] = (cols[f:t].copy(), cnt16[f:t].copy())
            r0 = r1
        rowsums = {a: int(rs32[a]) for a in np.flatnonzero(rs32)}
        # top-k operator: the owned heaps, in row ranges
        self.core.topk_owned_host(self.topk)
        heaps = {}
        for r0 in range(0, M, TOPK_ROWS_PER_RANGE):
            r1 = min(M, r0 + TOPK_ROWS_PER_RANGE)
            sz, vals, scores = self.core.copy_topk_range(r0, r1, self.topk)
            for j in np.flatnonzero(sz):
                heaps[r0 + int(j)] = (vals[j, :sz[j]].copy(), scores[j, :sz[j]].copy())
        return dict(timestamp=timestamp, rows=rows, rowsums=rowsums, heaps=heaps, observed=int(winfo.observed),
                    job_observed=int(info.observed), n_ranges=n_ranges, order=self.core.column_order(),
                    late=self.late)


# the watermarks of the job; subtask 1 does not receive those at SKIPPED_BY_1 (Flink's per-subtask minimum over
# its own input channels), so the two subtasks run process_watermark different numbers of times
MARKS = [999, 4000, 4999, 5500, 5998, 5999, 7000, (1 << 63) - 1]
SKIPPED_BY_1 = {1, 4, 6}


def _late_records(j):
    """Records arriving just after watermark MARKS[j] with timestamps at or below it (late on every subtask that
    received that watermark, and on the single-stream oracle): none after a watermark subtask 1 skipped, where
    they would not be late on subtask 1.  After 5500 they fall inside the open window [5000, 6000)."""
    if j in SKIPPED_BY_1 or MARKS[j] >= 7000:
        return []
    rng = np.random.default_rng(100 + j)
    w = MARKS[j]
    return [(int(u), int(i), int(t)) for u, i, t in
            zip(rng.integers(0, 2500, 40), rng.integers(0, 1000, 40), rng.integers(w - 499, w + 1, 40))]


def _worker(rank, world, port, out_dir, n_users, topk):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import pickle

    import torch
    import torch.distributed as dist

    import __graft_entry__

    pkg = __graft_entry__.load_package()
    from flink_cooccurrence_amd import sharding

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    up, it, M = _log(n_users)
    users, items, ts = _records(up, it)
    mine = users % world == rank  # keyBy(0)
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        sharding.init_comm_torch_ops(core)
        op = _OwnedSubtask(core, M, topk)
        out = None
        k, n = 0, len(users)
        for j, w in enumerate(MARKS):
            while k < n and ts[k] <= w:
                if mine[k]:
                    op.process_element(int(users[k]), int(items[k]), int(ts[k]))
                k += 1
            if rank == 1 and j in SKIPPED_BY_1:  # subtask 1's input channels hand it fewer watermarks
                continue
            r = op.process_watermark(w)
            if r is not None:
                assert out is None
                out = r
            for lu, li, lt in _late_records(j):  # late records after the watermark: dropped and counted
                if lu % world == rank:
                    op.process_element(lu, li, lt)
        assert out is not None and out["timestamp"] == 5999
        out["late"] = op.late  # (records after the window fired are late too)
        assert out["late"] == sum(1 for j in range(len(MARKS)) for lu, _, _ in _late_records(j) if lu % world == rank)
    with open(os.path.join(out_dir, f"rank{rank}.pkl"), "wb") as f:
        pickle.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


def test_owned_operators_call_sequence_vs_oracle(pkg, oracle, torch_cuda, tmp_path):
    import pickle

    import torch.multiprocessing as mp

    from tests._helpers import assert_row_topk, llr_atol

    world, n_users, topk = 2, 2500, 10
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), n_users, topk), nprocs=world, join=True)
    parts = [pickle.load(open(tmp_path / f"rank{r}.pkl", "rb")) for r in range(world)]
    up, it, M = _log(n_users)
    rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
    lens = np.diff(up)
    P = int(np.sum(lens * (lens - 1)))
    assert observed == P
    assert all(p["job_observed"] == P for p in parts) and sum(p["observed"] for p in parts) == P
    # the single-stream oracle (every record, every watermark): the same drops, the same accumulators
    users, items, ts = _records(up, it)
    ref = oracle.OracleStream(WINDOW_MS, topk=0)
    k, n, fired = 0, len(users), []
    for j, w in enumerate(MARKS):
        e = int(np.searchsorted(ts, w, side="right"))
        ref.process_elements(users[k:e], items[k:e], ts[k:e])
        k = e
        fired += ref.process_watermark(w)
        for lu, li, lt in _late_records(j):
            assert ref.process_element(lu, li, lt), "an injected record must be late for the oracle"
    assert [wo.ts for wo in fired] == [5999]
    acc = ref.counters()
    n_late = sum(len(_late_records(j)) for j in range(len(MARKS)))
    assert n_late > 0 and sum(p["late"] for p in parts) == acc["UserInteractionCounterLateElements"] == n_late
    assert acc["UserInteractionCounterObservedCooccurrences"] == P == fired[0].observed
    assert all(p["n_ranges"] > 10 for p in parts), "the forced range limit must split the copy-out"
    # rows: each row on exactly one subtask, int16 view of the closed form
    seen = {}
    for r, p in enumerate(parts):
        for a, (c, v16) in p["rows"].items():
            assert a not in seen, f"row {a} emitted by two subtasks"
            seen[a] = r
            want_c = cols[rp[a]:rp[a + 1]]
            assert np.array_equal(c, want_c), f"row {a}: columns"
            assert np.array_equal(v16, data[rp[a]:rp[a + 1]].astype(np.uint16).view(np.int16)), f"row {a}: counts"
    assert set(seen) == set(np.flatnonzero(np.diff(rp)).tolist())
    rs32 = rowsums.astype(np.int64).astype(np.uint64).astype(np.uint32).view(np.int32)
    got_rs = {}
    for p in parts:
        got_rs.update(p["rowsums"])
    assert got_rs == {int(a): int(rs32[a]) for a in np.flatnonzero(rs32)}
    # heaps: the oracle's rescorer over each row in the device's order (the tie order)
    r_obs = int(rs32.astype(np.int64).sum())  # the rescorer's long: the sum of the int row sums
    atol = llr_atol(r_obs)
    n_heaps = exact = 0
    for r, p in enumerate(parts):
        heap_rows = np.array(sorted(p["heaps"]), np.int32)
        assert set(heap_rows.tolist()) == {a for a, s in seen.items() if s == r}
        order = p["order"]
        hp = [0]
        hc, hv = [], []
        for a in heap_rows.tolist():
            c = cols[rp[a]:rp[a + 1]]
            o = np.argsort(order[c], kind="stable")
            hc.append(c[o])
            hv.append(data[rp[a]:rp[a + 1]][o].astype(np.uint16).view(np.int16))
            hp.append(hp[-1] + len(c))
        w_sz, w_v, w_sc = oracle.rows_topk(heap_rows, np.array(hp, np.int64), np.concatenate(hc), np.concatenate(hv),
                                           rs32, r_obs, topk)
        for j, a in enumerate(heap_rows.tolist()):
            v, sc = p["heaps"][a]
            want = [(int(w_v[j, i]), float(w_sc[j, i])) for i in range(int(w_sz[j]))]
            exact += assert_row_topk(len(v), v, sc, want, where=f"row {a}", atol=atol)
            n_heaps += 1
    print(f"{n_heaps} heaps, {exact} bit-identical")
    assert n_heaps == len(seen) and exact >= 0.9 * n_heaps


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch
