"""The JNI call sequence of the Java drop-in operators, replayed through the C-ABI (ctypes).

GpuNonSampledCooccurrenceRowsOperator (jvm/.../GpuNonSampledCooccurrenceRowsOperator.java) replaces the
pair emitter and both keyed window reducers (FlinkCooccurrences.java:65-74,135-157).  Per watermark it
calls, through cooc_jni.c:
  cooc_op_process_elements (the buffered records) -> cooc_op_process_watermark until nothing fires ->
  per fired window: cooc_copy_window_delta(rows, row_ptr, NULL...) -> cooc_copy_window_delta_range over
  row ranges of at most MAX_RANGE_ENTRIES entries (CoocWindowReader.java) -> cooc_copy_window_rowsums
and emits one Tuple2<Integer, Int2ShortOpenHashMap> per delta row and one Tuple2<Integer, Integer> per
non-zero int row-sum delta.  This test replays exactly that sequence (with a tiny range limit, so that
windows stream out in many ranges) and compares the records with what the reference's ItemRowAggregator
(ItemRowAggregator.java:26-31,50-56) and RowSumAggregator (RowSumAggregator.java:25-27,54-71) windows emit
for the same records and watermarks (oracle.OracleStream).  With p = 2 subtasks (users sharded by
keyBy(0)), the partial rows / row sums of the two handles are summed by the job's ItemRowMerge / IntSum
reducers (short and int wrap) and must equal the same records.  Needs an MI355X.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


class JniReplay:
    """cooc_jni.c + GpuNonSampledCooccurrenceRowsOperator, call for call."""

    def __init__(self, lib, n_items: int, window_ms: int, devices, subtask: int, max_range_entries: int):
        self.L, self.max_range = lib, max_range_entries
        from flink_cooccurrence_amd._lib import CoocConfig, check

        self.check = check
        cfg = CoocConfig(-1, n_items, 0, 0, window_ms, 0, 0)
        h = ctypes.c_void_p()
        devs = np.ascontiguousarray(devices, np.int32)
        check(lib.cooc_create_on(ctypes.byref(cfg), devs.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(devs),
                                 subtask, ctypes.byref(h)))
        self.h = h
        self.ranges = 0

    def close(self):
        self.L.cooc_destroy(self.h)

    @staticmethod
    def _p(a, t):
        return a.ctypes.data_as(ctypes.POINTER(t))

    def process_watermark(self, users, items, ts, watermark):
        """processWatermark: buffered records to the device, then every window the watermark closes."""
        from flink_cooccurrence_amd._lib import CoocWindowInfo

        u, i, t = (np.ascontiguousarray(users, np.int32), np.ascontiguousarray(items, np.int32),
                   np.ascontiguousarray(ts, np.int64))
        late = ctypes.c_int64()
        if len(u):
            self.check(self.L.cooc_op_process_elements(self.h, len(u), self._p(u, ctypes.c_int32), self._p(i, ctypes.c_int32),
                                                       self._p(t, ctypes.c_int64), ctypes.byref(late)), self.h)
        out = []
        while True:
            fired, info = ctypes.c_int32(), CoocWindowInfo()
            self.check(self.L.cooc_op_process_watermark(self.h, watermark, ctypes.byref(fired), ctypes.byref(info)), self.h)
            if not fired.value:
                return out, late.value
            out.append(self._emit_window(info))

    def _emit_window(self, info):
        """emitWindow + CoocWindowReader.forEachRow: ({item: {col: short}}, {item: int}, ts, observed)."""
        R = info.n_rows
        rows, row_ptr = np.zeros(R, np.int32), np.zeros(R + 1, np.int64)
        self.check(self.L.cooc_copy_window_delta(self.h, self._p(rows, ctypes.c_int32), self._p(row_ptr, ctypes.c_int64),
                                                 None, None, None), self.h)
        maps = {}
        r0 = 0
        while r0 < R:
            r1 = r0 + 1
            while r1 < R and row_ptr[r1 + 1] - row_ptr[r0] <= self.max_range:
                r1 += 1
            n = int(row_ptr[r1] - row_ptr[r0])
            cols, cnt16 = np.zeros(n, np.int32), np.zeros(n, np.int16)
            self.check(self.L.cooc_copy_window_delta_range(self.h, r0, r1, n, self._p(cols, ctypes.c_int32), None,
                                                           self._p(cnt16, ctypes.c_int16)), self.h)
            self.ranges += 1
            for r in range(r0, r1):
                s, e = int(row_ptr[r] - row_ptr[r0]), int(row_ptr[r + 1] - row_ptr[r0])
                maps[int(rows[r])] = dict(zip(cols[s:e].tolist(), cnt16[s:e].tolist()))
            r0 = r1
        items, d32 = np.zeros(R, np.int32), np.zeros(R, np.int32)
        self.check(self.L.cooc_copy_window_rowsums(self.h, self._p(items, ctypes.c_int32), None,
                                                   self._p(d32, ctypes.c_int32)), self.h)
        sums = {int(a): int(d) for a, d in zip(items, d32) if d != 0}  # RowSumAggregator.java:66
        return info.ts, maps, sums, info.observed


def _ref_records(w):
    """What the reference's two window functions emit for one fired oracle window."""
    maps = {}
    for r, a in enumerate(w.rows.tolist()):
        s, e = int(w.row_ptr[r]), int(w.row_ptr[r + 1])
        maps[a] = dict(zip(w.cols[s:e].tolist(), w.v16[s:e].tolist()))
    sums = {int(a): int(d) for a, d in zip(w.rs_items, w.rs_v32) if d != 0}
    return w.ts, maps, sums


def _merge(parts):
    """GpuCooccurrenceJob.ItemRowMerge (addTo: short wrap) and IntSum (int wrap) + filter(!= 0)."""
    maps, sums = {}, {}
    for m, s in parts:
        for a, row in m.items():
            acc = maps.setdefault(a, {})
            for b, v in row.items():
                acc[b] = int(np.int16(np.int64(acc.get(b, 0) + v).astype(np.int16)))
        for a, d in s.items():
            sums[a] = int(np.int64(sums.get(a, 0) + d).astype(np.int32))
    return maps, {a: d for a, d in sums.items() if d != 0}


@pytest.mark.parametrize("n_items,p", [(1000, 1), (1000, 2), (1_000_000, 1), (1_000_000, 2)])
def test_rows_operator_call_sequence_vs_reference_windows(pkg, oracle, torch_cuda, n_items, p):
    from flink_cooccurrence_amd import _lib, datagen

    L = _lib.load()
    d = datagen.config_c1(seed=8, U=800, M=n_items, mean=25.0)
    users, items, ts = datagen.to_records(d["user_ptr"], d["items"], d["ts"])
    # int16 wrap on the way: one heavy user repeating item 3 (C[3,3] = m (m - 1) > 32767 in one window)
    users = np.concatenate([users, np.full(200, 10**6, np.int32)])
    items = np.concatenate([items, np.full(200, 3, np.int32)])
    ts = np.concatenate([ts, np.full(200, int(ts[-1]), np.int64)])
    order = np.argsort(ts, kind="stable")
    users, items, ts = users[order], items[order], ts[order]
    ops = [JniReplay(L, n_items, 1000, [0], subtask=s, max_range_entries=257) for s in range(p)]
    ref = oracle.OracleStream(1000)
    by_ts, want, step = {}, [], 3000
    for lo in range(0, len(users), step):
        sl = slice(lo, lo + step)
        wm = int(ts[sl][-1]) - 1 if lo + step < len(users) else 2**63 - 1
        for s_, op in enumerate(ops):
            m = users[sl] % p == s_  # keyBy(0): the subtask of a user
            for w_ts, maps, sums, _ in op.process_watermark(users[sl][m], items[sl][m], ts[sl][m], wm)[0]:
                by_ts.setdefault(w_ts, []).append((maps, sums))
        ref.process_elements(users[sl], items[sl], ts[sl])
        want += [_ref_records(w) for w in ref.process_watermark(wm)]
    # the subtasks' partial rows of one window meet in the keyed reducers (p > 1)
    got = [(t,) + (_merge(parts) if p > 1 else parts[0]) for t, parts in sorted(by_ts.items())]
    assert len(got) == len(want) > 3
    for (gts, gm, gs), (wts, wm_, ws_) in zip(got, want):
        assert gts == wts
        assert gm == wm_, f"window {wts}: rows differ"
        assert gs == ws_, f"window {wts}: row sums differ"
    assert any(v < 0 for _, m, _ in want for row in m.values() for v in row.values()), "no int16 wrap exercised"
    assert all(op.ranges > len(got) for op in ops), "windows did not stream out in several ranges"
    for op in ops:
        op.close()


def test_delta_range_arguments(pkg, torch_cuda):
    """Ranges outside the window's delta rows fail with COOC_ERR_ARG (IllegalArgumentException)."""
    from flink_cooccurrence_amd import _lib

    op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1, "SECONDS", n_items=50, top_k=1)
    op.process_elements([1, 1, 2], [3, 4, 3], [10, 20, 30])
    (w,) = op.process_watermark(2000)
    L, h = _lib.load(), op.core._h
    n = len(w.rows)
    for r0, r1 in [(-1, 1), (2, 1), (0, n + 1)]:
        with pytest.raises(_lib.IllegalArgumentException):
            _lib.check(L.cooc_copy_window_delta_range(h, r0, r1, 0, None, None, None), h)
    _lib.check(L.cooc_copy_window_delta_range(h, 1, 1, 0, None, None, None), h)
    # a buffer smaller than the range (the JNI sizes its scratch from the Java length) is refused
    nb = int(w.row_ptr[n] - w.row_ptr[0])
    small = np.zeros(max(nb - 1, 0), np.int32)
    with pytest.raises(_lib.IllegalArgumentException):
        _lib.check(L.cooc_copy_window_delta_range(h, 0, n, nb - 1, small.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                  None, None), h)
    op.close()


class JniTopKReplay(JniReplay):
    """cooc_jni.c + GpuNonSampledCooccurrenceTopKOperator (the rescorer on the device too), call for call:
    create(topK) -> processElements -> processWatermark until nothing fires -> per fired window
    cooc_copy_window_topk(rows, sizes, values, scores) -> one IntDoublePriorityQueue per rescored row,
    rebuilt with add() in heap order (IntDoublePriorityQueue.java:132-137)."""

    def __init__(self, lib, n_items: int, window_ms: int, topk: int):
        from flink_cooccurrence_amd._lib import CoocConfig, check

        self.L, self.check, self.k = lib, check, topk
        cfg = CoocConfig(-1, n_items, topk, 0, window_ms, 0, 0)
        h = ctypes.c_void_p()
        devs = np.zeros(1, np.int32)
        check(lib.cooc_create_on(ctypes.byref(cfg), devs.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 1, 0,
                                 ctypes.byref(h)))
        self.h = h

    def _emit_window(self, info):
        """emitTopK: (ts, {item: [(value, score) in heap order]}) of one fired window."""
        from oracle import oracle

        n, k = info.n_topk, info.topk
        assert k == self.k
        rows, sizes = np.zeros(n, np.int32), np.zeros(n, np.int32)
        vals, scores = np.zeros(n * k, np.int32), np.zeros(n * k, np.float64)
        if n:
            self.check(self.L.cooc_copy_window_topk(self.h, self._p(rows, ctypes.c_int32), self._p(sizes, ctypes.c_int32),
                                                    self._p(vals, ctypes.c_int32), self._p(scores, ctypes.c_double)),
                       self.h)
        heaps = {}
        for r in range(n):
            q = oracle.PriorityQueue(k)  # topKReuse.reset(); add() in heap order
            for i in range(int(sizes[r])):
                q.add(int(vals[r * k + i]), float(scores[r * k + i]))
            got = q.entries()
            want = list(zip(vals[r * k:r * k + sizes[r]].tolist(), scores[r * k:r * k + sizes[r]].tolist()))
            assert [v for v, _ in got] == [v for v, _ in want], "add() in heap order changed the layout"
            heaps[int(rows[r])] = got
        return info.ts, heaps


@pytest.mark.parametrize("n_items", [1000, 1_000_000])
def test_topk_operator_call_sequence_vs_reference_rescorer(pkg, oracle, torch_cuda, n_items):
    """GpuNonSampledCooccurrenceTopKOperator's output -- one Tuple2<Integer, IntDoublePriorityQueue> per
    rescored item and window -- against the reference's ItemRowRescorerTwoInputStreamOperator fed by its own
    windows (oracle.OracleStream with topK: ItemRowRescorer...java:116-241), window by window, with an int16
    wrap on the way.  Heaps by the tolerance contract of SURVEY §8(a) (scores within 1e-6 relative, items
    strictly above the k-th score equal; the identical layout wherever every score agrees bit for bit)."""
    from flink_cooccurrence_amd import _lib, datagen

    from tests._helpers import assert_row_topk

    L, k = _lib.load(), 5
    d = datagen.config_c1(seed=12, U=700, M=n_items, mean=22.0)
    users, items, ts = datagen.to_records(d["user_ptr"], d["items"], d["ts"])
    users = np.concatenate([users, np.full(200, 10**6, np.int32)])
    items = np.concatenate([items, np.full(200, 3, np.int32)])
    ts = np.concatenate([ts, np.full(200, int(ts[-1]), np.int64)])
    order = np.argsort(ts, kind="stable")
    users, items, ts = users[order], items[order], ts[order]
    op = JniTopKReplay(L, n_items, 1000, k)
    ref = oracle.OracleStream(1000, topk=k)
    got, want, step = [], [], 2500
    for lo in range(0, len(users), step):
        sl = slice(lo, lo + step)
        wm = int(ts[sl][-1]) - 1 if lo + step < len(users) else 2**63 - 1
        got += op.process_watermark(users[sl], items[sl], ts[sl], wm)[0]
        ref.process_elements(users[sl], items[sl], ts[sl])
        want += ref.process_watermark(wm)
    assert len(got) == len(want) > 3
    n_heaps = 0
    for (gts, heaps), w in zip(got, want):
        assert gts == w.ts
        assert sorted(heaps) == sorted(w.topk_rows.tolist()), f"window {w.ts}: rescored items differ"
        for r, a in enumerate(w.topk_rows.tolist()):
            g = heaps[a]
            want_r = [(int(w.topk_values[r, i]), float(w.topk_scores[r, i])) for i in range(int(w.topk_sizes[r]))]
            assert_row_topk(len(g), [v for v, _ in g], [s for _, s in g], want_r, where=f"window {w.ts} row {a}")
            n_heaps += 1
    assert n_heaps > 100
    op.close()
