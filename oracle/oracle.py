"""Oracle for the co-occurrence hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module.  The product path (``flink-cooccurrence_amd``) never imports it and fails loudly
when its HIP library is missing; it has no CPU fallback.

Three independent restatements of the reference's non-sampled path:

1. ``OracleStream`` — ctypes wrapper of ``cooc_oracle.c``: the record-by-record restatement of
   NonSampledUserInteractionCounterOneInputStreamOperator.java:84-165, ItemRowAggregator.java:26-56,
   RowSumAggregator.java:25-71, ItemRowRescorerTwoInputStreamOperator.java:116-241,
   LogLikelihood.java:41-61 and IntDoublePriorityQueue.java:132-205.
2. ``closed_form`` — numpy/scipy ``C = A^T A - diag(colsum A)`` with A the user x item
   multiplicity matrix, row sums ``sum_u m_ua (n_u - 1)`` and observed ``sum_u n_u (n_u - 1)``
   (SURVEY.md §0.3).  Independent of (1): agreement of the two pins the literal expansion.
3. ``literal_python`` — pure-Python transliteration of NonSampled...java:129-161 for tiny logs.

Parity status: LLR and the heap are pinned by the reference's own KATs
(LogLikelihoodTest.java:14-16, IntDoublePriorityQueueTest.java:12-98).  No reference fixture pins
pair counts / row sums / windows and the Java reference cannot run here, so count parity is
"parity unpinned" by the reference; hand-derived micro-logs (tests/golden/micro_logs.json) and
the agreement of (1), (2) and (3) are what pin it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libcooc_oracle.so")
_lib = None

i32p = ctypes.POINTER(ctypes.c_int32)
i64p = ctypes.POINTER(ctypes.c_int64)
i16p = ctypes.POINTER(ctypes.c_int16)
f64p = ctypes.POINTER(ctypes.c_double)
u64p = ctypes.POINTER(ctypes.c_uint64)


def build() -> str:
    """Compile the C restatement (make in oracle/)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
        os.path.join(_HERE, "cooc_oracle.c")
    ):
        build()
    L = ctypes.CDLL(_LIB_PATH)
    vp = ctypes.c_void_p
    sig = {
        "oc_llr": (ctypes.c_double, [ctypes.c_int64] * 4),
        "oc_strict_log": (ctypes.c_double, [ctypes.c_double]),
        "oc_score_item": (ctypes.c_double, [ctypes.c_int16, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]),
        "oc_pq_create": (vp, [ctypes.c_int32]),
        "oc_pq_destroy": (None, [vp]),
        "oc_pq_size": (ctypes.c_int32, [vp]),
        "oc_pq_least_value": (ctypes.c_int32, [vp]),
        "oc_pq_least_score": (ctypes.c_double, [vp]),
        "oc_pq_reset": (None, [vp]),
        "oc_pq_add": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_double]),
        "oc_pq_update": (None, [vp, ctypes.c_int32, ctypes.c_double]),
        "oc_pq_entries": (None, [vp, i32p, f64p]),
        "oc_java_random_doubles": (None, [ctypes.c_int64, ctypes.c_int32, f64p]),
        "oc_java_random_next_int32": (None, [ctypes.c_int64, ctypes.c_int32, i32p]),
        "oc_java_random_ints": (None, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, i32p]),
        "oc_create": (vp, [ctypes.c_int64, ctypes.c_int32]),
        "oc_set_user_cut": (ctypes.c_int, [vp, ctypes.c_int32]),
        "oc_destroy": (None, [vp]),
        "oc_window_max_ts": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64]),
        "oc_process_element": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64]),
        "oc_process_elements": (ctypes.c_int64, [vp, ctypes.c_int64, i32p, i32p, i64p]),
        "oc_process_watermark": (ctypes.c_int32, [vp, ctypes.c_int64]),
        "oc_n_windows": (ctypes.c_int32, [vp]),
        "oc_window_ts": (ctypes.c_int64, [vp, ctypes.c_int32]),
        "oc_window_n_rows": (ctypes.c_int32, [vp, ctypes.c_int32]),
        "oc_window_nnz": (ctypes.c_int64, [vp, ctypes.c_int32]),
        "oc_window_observed": (ctypes.c_int64, [vp, ctypes.c_int32]),
        "oc_window_n_rowsums": (ctypes.c_int32, [vp, ctypes.c_int32]),
        "oc_window_n_topk": (ctypes.c_int32, [vp, ctypes.c_int32]),
        "oc_window_delta": (None, [vp, ctypes.c_int32, i32p, i64p, i32p, i64p, i16p]),
        "oc_window_rowsums": (None, [vp, ctypes.c_int32, i32p, i64p, i32p]),
        "oc_window_topk": (None, [vp, ctypes.c_int32, i32p, i32p, i32p, f64p]),
        "oc_counters": (None, [vp, i64p]),
        "oc_global_n_rows": (ctypes.c_int32, [vp]),
        "oc_global_nnz": (ctypes.c_int64, [vp]),
        "oc_global_rows": (None, [vp, i32p, i64p, i32p, i64p, i16p]),
        "oc_global_n_rowsums": (ctypes.c_int32, [vp]),
        "oc_global_rowsums": (None, [vp, i32p, i32p, i64p]),
        "oc_batch_dense": (ctypes.c_int64, [ctypes.c_int64, i64p, i32p, ctypes.c_int32, i64p, i64p]),
        "oc_count_batch_mt": (ctypes.c_int64, [ctypes.c_int64, i64p, i32p, ctypes.c_int32, ctypes.c_int32, i64p]),
        "oc_count_batch_mt_rows": (ctypes.c_int64, [ctypes.c_int64, i64p, i32p, ctypes.c_int32, ctypes.c_int32, i64p,
                                                    u64p, i64p, i64p]),
        "oc_row_checksums": (ctypes.c_int64, [ctypes.c_int64, i64p, i32p, ctypes.c_int32, ctypes.c_int32, i64p,
                                              u64p, i64p, i64p]),
        "oc_rows_topk": (None, [ctypes.c_int64, i32p, i64p, i32p, ctypes.POINTER(ctypes.c_int16), i32p, ctypes.c_int64,
                                ctypes.c_int32, ctypes.c_int32, i32p, i32p, ctypes.POINTER(ctypes.c_double)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


# ---------------------------------------------------------------------------------------------
# LogLikelihood / IntDoublePriorityQueue / java.util.Random restatements
# ---------------------------------------------------------------------------------------------
def strict_log(x: float) -> float:
    """Java's StrictMath.log (fdlibm 5.3 __ieee754_log), the log of the LLR restatement."""
    return lib().oc_strict_log(x)


def llr(k11: int, k12: int, k21: int, k22: int) -> float:
    """LogLikelihood.logLikelihoodRatio, LogLikelihood.java:41-57."""
    return lib().oc_llr(k11, k12, k21, k22)


def score_item(k11_i16: int, item_row_sum: int, other_row_sum: int, observed: int) -> float:
    """ItemRowRescorerTwoInputStreamOperator.scoreItem, :230-241."""
    return lib().oc_score_item(k11_i16, item_row_sum, other_row_sum, observed)


def rows_topk(row_items, row_ptr, cols, cnt16, rs32, observed: int, k: int, n_threads: int = 1):
    """The rescorer's heaps of the given rows (ItemRowRescorer...java:195-223), entries fed in the order
    given: row j is item row_items[j], entries [row_ptr[j], row_ptr[j+1]) of cols / cnt16 (int16 counts);
    rs32 = every item's int row sum; observed = the rescorer's long.  -> (sizes [n], values [n, k],
    scores [n, k]) in IntDoublePriorityQueue order (positions 1..size)."""
    ri = np.ascontiguousarray(row_items, np.int32)
    rp = np.ascontiguousarray(row_ptr, np.int64)
    c = np.ascontiguousarray(cols, np.int32)
    v = np.ascontiguousarray(cnt16, np.int16)
    rs = np.ascontiguousarray(rs32, np.int32)
    n = len(ri)
    sizes = np.zeros(n, np.int32)
    vals = np.zeros((n, k), np.int32)
    scores = np.zeros((n, k), np.float64)
    lib().oc_rows_topk(n, _p(ri, i32p), _p(rp, i64p), _p(c, i32p), v.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)),
                       _p(rs, i32p), int(observed), int(k), int(n_threads), _p(sizes, i32p), _p(vals, i32p),
                       scores.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return sizes, vals, scores


class PriorityQueue:
    """IntDoublePriorityQueue.java restated in C (1-based Lucene min-heap)."""

    def __init__(self, max_size: int):
        if max_size < 1:
            raise ValueError("maxSize not positive")  # IntDoublePriorityQueue.java:70-72
        self._q = lib().oc_pq_create(max_size)
        self.max_size = max_size

    def __del__(self):
        if getattr(self, "_q", None):
            lib().oc_pq_destroy(self._q)
            self._q = None

    def size(self) -> int:
        return lib().oc_pq_size(self._q)

    def least_value(self) -> int:
        return lib().oc_pq_least_value(self._q)

    def least_score(self) -> float:
        return lib().oc_pq_least_score(self._q)

    def reset(self) -> None:
        lib().oc_pq_reset(self._q)

    def add(self, value: int, score: float) -> None:
        if lib().oc_pq_add(self._q, value, score) != 0:
            raise IndexError("ArrayIndexOutOfBoundsException")  # Java's behaviour at :133-134

    def update(self, value: int, score: float) -> None:
        lib().oc_pq_update(self._q, value, score)

    def entries(self):
        n = self.size()
        v = np.zeros(n, np.int32)
        s = np.zeros(n, np.float64)
        lib().oc_pq_entries(self._q, _p(v, i32p), _p(s, f64p))
        return list(zip(v.tolist(), s.tolist()))


def java_random_doubles(seed: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.float64)
    lib().oc_java_random_doubles(seed, n, _p(out, f64p))
    return out


def java_random_next_int32(seed: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.int32)
    lib().oc_java_random_next_int32(seed, n, _p(out, i32p))
    return out


def java_random_ints(seed: int, bound: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.int32)
    lib().oc_java_random_ints(seed, bound, n, _p(out, i32p))
    return out


def window_max_ts(ts: int, size: int) -> int:
    return lib().oc_window_max_ts(ts, size)


# ---------------------------------------------------------------------------------------------
# Streaming restatement: processElement / processWatermark and every fired window's outputs
# ---------------------------------------------------------------------------------------------
@dataclass
class WindowOutput:
    ts: int
    rows: np.ndarray       # int32 [R] ascending item ids with a delta row
    row_ptr: np.ndarray    # int64 [R+1]
    cols: np.ndarray       # int32 [nnz] ascending within a row
    exact: np.ndarray      # int64 [nnz]
    v16: np.ndarray        # int16 [nnz]  (Int2ShortOpenHashMap values)
    rs_items: np.ndarray   # int32 items with non-zero exact row-sum delta
    rs_exact: np.ndarray   # int64
    rs_v32: np.ndarray     # int32 (RowSumAggregator int accumulation)
    observed: int          # ObservedCooccurrences accumulator delta
    topk_rows: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    topk_sizes: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    topk_values: np.ndarray = field(default_factory=lambda: np.zeros((0, 0), np.int32))
    topk_scores: np.ndarray = field(default_factory=lambda: np.zeros((0, 0), np.float64))


class OracleStream:
    """Record-by-record restatement of the skip-cuts job from the keyBy(user) edge onwards."""

    def __init__(self, window_size_ms: int, topk: int = 0, user_cut: int = 0):
        self._s = lib().oc_create(window_size_ms, topk)
        if not self._s:
            raise ValueError("bad window size / topk")
        if lib().oc_set_user_cut(self._s, user_cut):
            raise ValueError("userCut must be a Java short >= 0")
        self.topk = topk
        self._read = 0

    def __del__(self):
        if getattr(self, "_s", None):
            lib().oc_destroy(self._s)
            self._s = None

    def process_element(self, user: int, item: int, ts: int) -> bool:
        """Returns True when the element was late and dropped (NonSampled...java:89-91)."""
        return bool(lib().oc_process_element(self._s, user, item, ts))

    def process_elements(self, users, items, ts) -> int:
        u = np.ascontiguousarray(users, np.int32)
        i = np.ascontiguousarray(items, np.int32)
        t = np.ascontiguousarray(ts, np.int64)
        return lib().oc_process_elements(self._s, len(u), _p(u, i32p), _p(i, i32p), _p(t, i64p))

    def process_watermark(self, wm: int) -> list[WindowOutput]:
        lib().oc_process_watermark(self._s, wm)
        return self._drain()

    def _drain(self) -> list[WindowOutput]:
        L = lib()
        out = []
        n = L.oc_n_windows(self._s)
        for w in range(self._read, n):
            R = L.oc_window_n_rows(self._s, w)
            nnz = L.oc_window_nnz(self._s, w)
            rows = np.zeros(R, np.int32)
            row_ptr = np.zeros(R + 1, np.int64)
            cols = np.zeros(nnz, np.int32)
            exact = np.zeros(nnz, np.int64)
            v16 = np.zeros(nnz, np.int16)
            L.oc_window_delta(self._s, w, _p(rows, i32p), _p(row_ptr, i64p), _p(cols, i32p), _p(exact, i64p),
                              _p(v16, i16p))
            nr = L.oc_window_n_rowsums(self._s, w)
            rs_items = np.zeros(nr, np.int32)
            rs_exact = np.zeros(nr, np.int64)
            rs_v32 = np.zeros(nr, np.int32)
            L.oc_window_rowsums(self._s, w, _p(rs_items, i32p), _p(rs_exact, i64p), _p(rs_v32, i32p))
            wo = WindowOutput(L.oc_window_ts(self._s, w), rows, row_ptr, cols, exact, v16, rs_items, rs_exact,
                              rs_v32, L.oc_window_observed(self._s, w))
            nt = L.oc_window_n_topk(self._s, w)
            if self.topk > 0:
                tr = np.zeros(nt, np.int32)
                ts_ = np.zeros(nt, np.int32)
                tv = np.zeros((nt, self.topk), np.int32)
                tsc = np.zeros((nt, self.topk), np.float64)
                L.oc_window_topk(self._s, w, _p(tr, i32p), _p(ts_, i32p), _p(tv, i32p), _p(tsc, f64p))
                wo.topk_rows, wo.topk_sizes, wo.topk_values, wo.topk_scores = tr, ts_, tv, tsc
            out.append(wo)
        self._read = n
        return out

    def counters(self) -> dict:
        a = np.zeros(5, np.int64)
        lib().oc_counters(self._s, _p(a, i64p))
        return {
            "UserInteractionCounterLateElements": int(a[0]),
            "UserInteractionCounterObservedCooccurrences": int(a[1]),
            "RowSumProcessWindowRowSum": int(a[2]),
            "ItemRowRescorerRescoredItems": int(a[3]),
            "rescorer_observed": int(a[4]),
        }

    def global_rows(self):
        L = lib()
        R = L.oc_global_n_rows(self._s)
        nnz = L.oc_global_nnz(self._s)
        rows = np.zeros(R, np.int32)
        row_ptr = np.zeros(R + 1, np.int64)
        cols = np.zeros(nnz, np.int32)
        exact = np.zeros(nnz, np.int64)
        v16 = np.zeros(nnz, np.int16)
        L.oc_global_rows(self._s, _p(rows, i32p), _p(row_ptr, i64p), _p(cols, i32p), _p(exact, i64p), _p(v16, i16p))
        return rows, row_ptr, cols, exact, v16

    def global_rowsums(self):
        L = lib()
        n = L.oc_global_n_rowsums(self._s)
        items = np.zeros(n, np.int32)
        v32 = np.zeros(n, np.int32)
        exact = np.zeros(n, np.int64)
        L.oc_global_rowsums(self._s, _p(items, i32p), _p(v32, i32p), _p(exact, i64p))
        return items, v32, exact


# ---------------------------------------------------------------------------------------------
# One-window batch forms (the stateless device entry point's contract)
# ---------------------------------------------------------------------------------------------
def batch_dense(user_ptr: np.ndarray, items: np.ndarray, n_items: int):
    """Literal expansion (C) of one window over empty histories -> dense int64 counts."""
    user_ptr = np.ascontiguousarray(user_ptr, np.int64)
    items = np.ascontiguousarray(items, np.int32)
    counts = np.zeros((n_items, n_items), np.int64)
    rowsums = np.zeros(n_items, np.int64)
    obs = lib().oc_batch_dense(len(user_ptr) - 1, _p(user_ptr, i64p), _p(items, i32p), n_items,
                               _p(counts, i64p), _p(rowsums, i64p))
    return counts, rowsums, int(obs)


def count_batch_mt(user_ptr: np.ndarray, items: np.ndarray, n_items: int, n_threads: int):
    """Multithreaded record-by-record restatement of one window (threads own rows a mod n_threads):
    -> (distinct keys, ordered pairs).  The CPU baseline of bench.py."""
    up = np.ascontiguousarray(user_ptr, np.int64)
    it = np.ascontiguousarray(items, np.int32)
    pairs = np.zeros(1, np.int64)
    nnz = lib().oc_count_batch_mt(len(up) - 1, _p(up, i64p), _p(it, i32p), n_items, n_threads, _p(pairs, i64p))
    return int(nnz), int(pairs[0])


@dataclass
class RowChecks:
    """Per-row exactness fingerprint of a count matrix: checksum = sum over the row's keys of
    splitmix64(col << 32 ^ exact count) mod 2^64 (row_key_hash; the library's cooc_verify_batch
    computes the same), distinct keys and the sum of the counts; plus the totals."""
    checksum: np.ndarray  # uint64 [n_items]
    nnz: np.ndarray       # int64 [n_items]
    rowsum: np.ndarray    # int64 [n_items]
    distinct: int
    pairs: int


def _row_checks(fn, user_ptr, items, n_items: int, n_threads: int) -> RowChecks:
    up = np.ascontiguousarray(user_ptr, np.int64)
    it = np.ascontiguousarray(items, np.int32)
    cs = np.zeros(n_items, np.uint64)
    nz = np.zeros(n_items, np.int64)
    rs = np.zeros(n_items, np.int64)
    pairs = np.zeros(1, np.int64)
    nnz = fn(len(up) - 1, _p(up, i64p), _p(it, i32p), n_items, n_threads, _p(pairs, i64p), _p(cs, u64p), _p(nz, i64p),
             _p(rs, i64p))
    return RowChecks(cs, nz, rs, int(nnz), int(pairs[0]))


def count_batch_mt_rows(user_ptr, items, n_items: int, n_threads: int) -> RowChecks:
    """count_batch_mt (the record-by-record restatement, NonSampled...java:129-161 into
    Int2ShortOpenHashMap restatements) with its per-row fingerprints."""
    return _row_checks(lib().oc_count_batch_mt_rows, user_ptr, items, n_items, n_threads)


def row_checksums(user_ptr, items, n_items: int, n_threads: int) -> RowChecks:
    """The same fingerprints from the closed form (C = A^T A - diag(colsum A), row by row with a dense
    accumulator per thread): fast enough for the benchmark's 3.4e10-pair shard."""
    return _row_checks(lib().oc_row_checksums, user_ptr, items, n_items, n_threads)


def row_key_hash(cols, counts) -> np.ndarray:
    """splitmix64((col << 32) ^ count) per entry (uint64), the checksum term of RowChecks."""
    with np.errstate(over="ignore"):
        x = (np.asarray(cols, np.int64).astype(np.uint64) << np.uint64(32)) ^ np.asarray(counts, np.int64).astype(np.uint64)
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def csr_row_checks(row_ptr, cols, counts) -> RowChecks:
    """RowChecks of a sorted CSR (e.g. closed_form's)."""
    rp = np.asarray(row_ptr, np.int64)
    M = len(rp) - 1
    rows = np.repeat(np.arange(M), np.diff(rp))
    h = row_key_hash(cols, counts)
    cs = np.zeros(M, np.uint64)
    np.add.at(cs, rows, h)
    rs = np.zeros(M, np.int64)
    np.add.at(rs, rows, np.asarray(counts, np.int64))
    return RowChecks(cs, np.diff(rp), rs, int(rp[-1]), int(rs.sum()))


def cut_csr(user_ptr: np.ndarray, items: np.ndarray, user_cut: int):
    """The first user_cut items of every user (kMax, one window over empty histories)."""
    user_ptr = np.asarray(user_ptr, np.int64)
    lens = np.minimum(np.diff(user_ptr), user_cut)
    keep = np.concatenate([np.arange(user_ptr[u], user_ptr[u] + lens[u]) for u in range(len(lens))]
                          + [np.zeros(0, np.int64)])
    return np.concatenate([[0], np.cumsum(lens)]).astype(np.int64), np.asarray(items)[keep].astype(np.int32)


def closed_form(user_ptr: np.ndarray, items: np.ndarray, n_items: int):
    """C = A^T A - diag(colsum A) as a sorted CSR (scipy), row sums and observed."""
    import scipy.sparse as sp

    user_ptr = np.asarray(user_ptr, np.int64)
    items = np.asarray(items, np.int64)
    U = len(user_ptr) - 1
    lens = np.diff(user_ptr)
    users = np.repeat(np.arange(U, dtype=np.int64), lens)
    A = sp.csr_matrix((np.ones(len(items), np.int64), (users, items)), shape=(U, n_items))
    A.sum_duplicates()
    colsum = np.asarray(A.sum(axis=0)).ravel().astype(np.int64)
    C = (A.T @ A).tocsr()
    C = C - sp.diags(colsum, format="csr")
    C.eliminate_zeros()
    C.sort_indices()
    rowsums = np.zeros(n_items, np.int64)
    np.add.at(rowsums, items, np.repeat(lens - 1, lens))
    observed = int(np.sum(lens * (lens - 1)))
    return C.indptr.astype(np.int64), C.indices.astype(np.int32), C.data.astype(np.int64), rowsums, observed


def literal_python(histories: list[list[int]], user_cut: int = 0):
    """Pure-Python NonSampled...java:129-161 over per-user item lists (tiny inputs only).
    user_cut > 0: UserInteractionCounter...java:168-205, an interaction is expanded only while the
    user has fewer than user_cut accepted ones (later ones dropped, no reservoir)."""
    counts: dict[tuple[int, int], int] = {}
    rowsums: dict[int, int] = {}
    observed = 0
    for items in histories:
        history: list[int] = []
        for item in items:
            size = len(history)
            if user_cut > 0 and size >= user_cut:
                continue
            if size > 0:
                for o in history:
                    counts[(item, o)] = counts.get((item, o), 0) + 1
                rowsums[item] = rowsums.get(item, 0) + size
                for o in history:
                    counts[(o, item)] = counts.get((o, item), 0) + 1
                    rowsums[o] = rowsums.get(o, 0) + 1
                observed += 2 * size
            history.append(item)
    return counts, rowsums, observed


def to_i16(x):
    return np.asarray(x, np.int64).astype(np.uint16).view(np.int16)


def to_i32(x):
    return np.asarray(x, np.int64).astype(np.uint32).view(np.int32)
