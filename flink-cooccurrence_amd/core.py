"""Host-side mirror of the reference's operator interface over the C-ABI.

The reference (Java, Flink 1.3.2) cannot be built here, so the host side above the C-ABI mirrors its
operator surface with the same names, argument meaning and error behaviour:

* ``NonSampledUserInteractionCounterOneInputStreamOperator`` —
  NonSampledUserInteractionCounterOneInputStreamOperator.java:31-178 (constructor ``(windowSize,
  windowUnit)`` :61, ``processElement`` :84-110, ``onEventTime`` :113-165) fused with the two window
  aggregators it feeds (ItemRowAggregator.java:15-57, RowSumAggregator.java:15-72) and the rescorer
  (ItemRowRescorerTwoInputStreamOperator.java:22-246, constructor ``(short topK)`` :51-56).
  ``process_watermark`` returns the fired windows' outputs: per-window delta rows (the
  ``Tuple2<Integer, Int2ShortOpenHashMap>`` records), row-sum updates (``Tuple2<Integer,Integer>``)
  and the top-k queues (``Tuple2<Integer, IntDoublePriorityQueue>``).
* ``CooccurrenceCore`` — one C-ABI context: the stateless one-window batch (``count``,
  ``count_device``) and the streaming window API (``submit_batch`` / ``finish_window``).

Every compute call goes through libcooc_hip.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import (CoocCommOps, CoocConfig, CoocDeviceResult, CoocOwnedInfo, CoocWindowInfo, check, f64p, i16p, i32p,
                   i64p, u32p)

# Configuration.java:160-182 window units -> milliseconds (Time.of(size, unit).toMilliseconds())
_UNIT_MS = {"MILLISECONDS": 1, "SECONDS": 1000, "MINUTES": 60_000, "HOURS": 3_600_000, "DAYS": 86_400_000}


def window_size_ms(size: int, unit: str = "MILLISECONDS") -> int:
    u = unit.upper()
    if u not in _UNIT_MS:
        raise _lib.IllegalArgumentException(_lib.COOC_ERR_ARG, f"Unrecognized window unit {unit}")  # :176-177
    return int(size) * _UNIT_MS[u]


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t) if a is not None else None


def _stream_arg(stream, tensor):
    """The HIP stream a device-tensor entry point runs on: the caller's, else torch's current stream
    on the tensor's device, so that the library's kernels are ordered after the work that produced
    the inputs and before the work that consumes the outputs (cooc.h, stream contract)."""
    if stream is not None:
        return ctypes.c_void_p(int(stream))
    import torch

    if getattr(tensor, "is_cuda", False):
        return ctypes.c_void_p(torch.cuda.current_stream(tensor.device).cuda_stream)
    return None


@dataclass
class BatchResult:
    """C of one window over empty histories, as a packed CSR over all n_items rows."""
    row_ptr: np.ndarray   # int64 [M+1]
    cols: np.ndarray      # int32 [nnz], ascending within a row
    cnt: np.ndarray       # uint32 [nnz] exact
    cnt16: np.ndarray     # int16 [nnz]   Int2ShortOpenHashMap view
    rowsum: np.ndarray    # int64 [M] exact
    rowsum32: np.ndarray  # int32 [M]     Java int view
    observed: int         # sum_u n_u (n_u - 1)


@dataclass
class WindowResult:
    """One fired window's observable outputs (same layout as oracle.WindowOutput)."""
    ts: int
    rows: np.ndarray
    row_ptr: np.ndarray
    cols: np.ndarray
    exact: np.ndarray
    v16: np.ndarray
    rs_items: np.ndarray
    rs_exact: np.ndarray
    rs_v32: np.ndarray
    observed: int
    topk_rows: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    topk_sizes: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    topk_values: np.ndarray = field(default_factory=lambda: np.zeros((0, 0), np.int32))
    topk_scores: np.ndarray = field(default_factory=lambda: np.zeros((0, 0), np.float64))


class CooccurrenceCore:
    """One context of the C-ABI (one Flink subtask)."""

    def __init__(self, n_items: int, topk: int = 0, window_size_ms: int = 1000, device: int = -1,
                 exact_scores: bool = False, output: str = "auto", planner: str = "auto", user_cut: int = 0,
                 devices=None, subtask: int = 0, column_order: bool = False, any_order: bool = False):
        """output: layout of count_device results: "auto", "csr" (padded CSR) or "dense" (n_items^2).
        planner: "auto" (the batch planner below 40,320 items, the large-universe planner above), "large"
        (the large-universe planner at any n_items; "general" is an alias) or "sort" (large, with every
        whole row through the sort + segmented-reduce path: packed 64-bit pair keys, radix sort, runs).
        user_cut: kMax, 0 = off; else only the first user_cut interactions of every user are expanded
        (UserInteractionCounter...java:168-205, the deterministic branch; later ones are dropped).
        column_order: COOC_FLAG_COLUMN_ORDER (device rows of the large-universe path in id order instead of the
        renumbered order: the batch's 16,384 most frequent items first, in id order, then the rest in id order;
        the renumbering is skipped when 15/16 of those hot items already have ids below 16,384).
        any_order: COOC_FLAG_ANY_ORDER (large-universe batch rows in no particular order: the LDS hash chunks skip
        their column ranking; host copies still come out sorted)."""
        L = _lib.load()
        flags = _lib.COOC_FLAG_EXACT_SCORES if exact_scores else 0
        if output not in ("auto", "csr", "dense"):
            raise _lib.IllegalArgumentException(_lib.COOC_ERR_ARG, f"unknown output layout {output!r}")
        flags |= {"auto": 0, "csr": _lib.COOC_FLAG_OUTPUT_CSR, "dense": _lib.COOC_FLAG_OUTPUT_DENSE}[output]
        if planner not in ("auto", "general", "large", "sort"):
            raise _lib.IllegalArgumentException(_lib.COOC_ERR_ARG, f"unknown planner {planner!r}")
        flags |= _lib.COOC_FLAG_GENERAL_PLANNER if planner != "auto" else 0
        flags |= _lib.COOC_FLAG_SORT_ROWS if planner == "sort" else 0
        flags |= _lib.COOC_FLAG_COLUMN_ORDER if column_order else 0
        flags |= _lib.COOC_FLAG_ANY_ORDER if any_order else 0
        cfg = CoocConfig(device, n_items, topk, flags, window_size_ms, user_cut, 0)
        h = ctypes.c_void_p()
        if devices is None:
            check(L.cooc_create(ctypes.byref(cfg), ctypes.byref(h)), None)
        else:  # create(cfg{devices[]}): this subtask's GPU is devices[subtask % len(devices)]
            devs = np.ascontiguousarray(devices, np.int32)
            check(L.cooc_create_on(ctypes.byref(cfg), _p(devs, i32p), len(devs), int(subtask), ctypes.byref(h)), None)
        self._h = h
        self.n_items = n_items
        self.topk = topk
        self.device = int(device) if devices is None else int(np.asarray(devices)[subtask % len(devices)])
        self.comm_world = 0  # > 0 once comm_init / comm_init_ops joined a communicator

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().cooc_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- stateless one-window batch -------------------------------------------------------------
    def count_device(self, user_ptr, items, stream=None) -> CoocDeviceResult:
        """user_ptr: int64 device tensor [U+1] (user_ptr[0] == 0); items: int32 device tensor."""
        res = CoocDeviceResult()
        n_users = int(user_ptr.numel()) - 1
        check(_lib.load().cooc_count_device(self._h, n_users, ctypes.c_void_p(user_ptr.data_ptr()),
                                            ctypes.c_void_p(items.data_ptr()), int(items.numel()),
                                            _stream_arg(stream, items), ctypes.byref(res)), self._h)
        return res

    def item_counts(self, items, out=None, stream=None):
        """Item frequencies of a device int32 tensor -> int64 device tensor [n_items] (cooc_item_counts)."""
        import torch

        if out is None:
            out = torch.empty(self.n_items, dtype=torch.int64, device=items.device)
        check(_lib.load().cooc_item_counts(self._h, ctypes.c_void_p(items.data_ptr()) if items.numel() else None,
                                           int(items.numel()), ctypes.c_void_p(out.data_ptr()),
                                           _stream_arg(stream, out)), self._h)
        return out

    def count_device_owned(self, user_ptr, items, owner, part: int, item_counts, n_total: int,
                           stream=None) -> CoocDeviceResult:
        """Rows a with owner[a] == part over every user given (multi-GPU, n_items >= 40,320).
        owner: int32 device tensor [n_items]; item_counts: int64 device tensor [n_items] of the
        global log (n_total interactions)."""
        res = CoocDeviceResult()
        n_users = int(user_ptr.numel()) - 1
        check(_lib.load().cooc_count_device_owned(
            self._h, n_users, ctypes.c_void_p(user_ptr.data_ptr()), ctypes.c_void_p(items.data_ptr()),
            int(items.numel()), ctypes.c_void_p(owner.data_ptr()), int(part), ctypes.c_void_p(item_counts.data_ptr()),
            int(n_total), _stream_arg(stream, items), ctypes.byref(res)), self._h)
        return res

    def count(self, user_ptr, items) -> BatchResult:
        up = np.ascontiguousarray(user_ptr, np.int64)
        it = np.ascontiguousarray(items, np.int32)
        info = CoocWindowInfo()
        L = _lib.load()
        check(L.cooc_count_host(self._h, len(up) - 1, _p(up, i64p), _p(it, i32p), ctypes.byref(info)), self._h)
        return self.copy_batch(info.nnz, info.observed)

    def copy_batch(self, nnz: int, observed: int) -> BatchResult:
        M = self.n_items
        rp = np.zeros(M + 1, np.int64)
        cols = np.zeros(nnz, np.int32)
        cnt = np.zeros(nnz, np.uint32)
        cnt16 = np.zeros(nnz, np.int16)
        rs = np.zeros(M, np.int64)
        rs32 = np.zeros(M, np.int32)
        check(_lib.load().cooc_copy_batch(self._h, _p(rp, i64p), _p(cols, i32p), _p(cnt, u32p), _p(cnt16, i16p),
                                          _p(rs, i64p), _p(rs32, i32p)), self._h)
        return BatchResult(rp, cols, cnt, cnt16, rs, rs32, int(observed))

    def column_order(self) -> np.ndarray:
        """cooc_copy_column_order: the position of every column in the last batch's device row order (its
        top-k iteration order): the descending-frequency rank after the large-universe relabel, else the
        column id."""
        out = np.zeros(self.n_items, np.int32)
        check(_lib.load().cooc_copy_column_order(self._h, _p(out, i32p)), self._h)
        return out

    def topk_batch(self, topk: int, exact_scores: bool = False, stream=None):
        """LLR top-k of every row of the last batch -> (sizes [M], values [M, k], scores [M, k])."""
        L = _lib.load()
        check(L.cooc_topk_batch(self._h, topk, _lib.COOC_FLAG_EXACT_SCORES if exact_scores else 0,
                                None if stream is None else ctypes.c_void_p(int(stream))), self._h)
        M = self.n_items
        sizes = np.zeros(M, np.int32)
        vals = np.zeros((M, topk), np.int32)
        scores = np.zeros((M, topk), np.float64)
        check(L.cooc_copy_topk_batch(self._h, _p(sizes, i32p), _p(vals, i32p), _p(scores, f64p)), self._h)
        return sizes, vals, scores

    def topk_batch_device(self, topk: int, sizes, values, scores, rowsum_global=None, exact_scores: bool = False,
                          stream=None) -> None:
        """LLR top-k of every row of the last batch into device tensors (sizes int32 [M], values int32
        [M, k], scores float64 [M, k]) on torch's current stream.  rowsum_global (int64 device [M]):
        the all-reduced row sums of a multi-GPU run (rows not owned here come out with size 0)."""
        check(_lib.load().cooc_topk_batch_device(
            self._h, topk, _lib.COOC_FLAG_EXACT_SCORES if exact_scores else 0,
            None if rowsum_global is None else ctypes.c_void_p(rowsum_global.data_ptr()),
            ctypes.c_void_p(sizes.data_ptr()), ctypes.c_void_p(values.data_ptr()), ctypes.c_void_p(scores.data_ptr()),
            _stream_arg(stream, sizes)), self._h)

    def llr(self, k4) -> np.ndarray:
        """LogLikelihood.logLikelihoodRatio of each (k11, k12, k21, k22) row, on the device."""
        k = np.ascontiguousarray(k4, np.int64).reshape(-1, 4)
        out = np.zeros(len(k), np.float64)
        check(_lib.load().cooc_llr(self._h, len(k), _p(k, i64p), _p(out, f64p)), self._h)
        return out

    def topk_items(self, items, k: int, exact_scores: bool = False):
        """topk(handle, items[], k) of SURVEY §8(b): the top-k of the given rows of the last batch ->
        (sizes [n], values [n, k], scores [n, k]), heap layout as topk_batch."""
        its = np.ascontiguousarray(items, np.int32)
        n = len(its)
        sizes = np.zeros(n, np.int32)
        vals = np.zeros((n, k), np.int32)
        scores = np.zeros((n, k), np.float64)
        check(_lib.load().cooc_topk_items(self._h, k, _lib.COOC_FLAG_EXACT_SCORES if exact_scores else 0, n,
                                          _p(its, i32p), _p(sizes, i32p), _p(vals, i32p), _p(scores, f64p)), self._h)
        return sizes, vals, scores

    # ---- sharding layer (owner-partitioned exchange of partial rows) -----------------------------
    def partition_plan(self, n_parts: int) -> np.ndarray:
        out = np.zeros(n_parts, np.int64)
        check(_lib.load().cooc_partition_plan(self._h, n_parts, _p(out, i64p)), self._h)
        return out

    def partition_pack(self, n_parts: int, row_nnz, entries, stream=None) -> None:
        """row_nnz: int32 device tensor [n_items]; entries: int64 device tensor [sum of the plan]."""
        check(_lib.load().cooc_partition_pack(self._h, n_parts, ctypes.c_void_p(row_nnz.data_ptr()),
                                              ctypes.c_void_p(entries.data_ptr()) if entries.numel() else None,
                                              _stream_arg(stream, row_nnz)), self._h)

    def copy_rowsum_device(self, rowsum, stream=None) -> None:
        check(_lib.load().cooc_copy_rowsum_device(self._h, ctypes.c_void_p(rowsum.data_ptr()),
                                                  _stream_arg(stream, rowsum)),
              self._h)

    def merge_partitions(self, n_parts: int, part: int, recv_row_nnz, recv_entries, rowsum_global=None,
                         stream=None) -> CoocDeviceResult:
        res = CoocDeviceResult()
        check(_lib.load().cooc_merge_partitions(
            self._h, n_parts, part, ctypes.c_void_p(recv_row_nnz.data_ptr()),
            ctypes.c_void_p(recv_entries.data_ptr()) if recv_entries.numel() else None,
            None if rowsum_global is None else ctypes.c_void_p(rowsum_global.data_ptr()),
            _stream_arg(stream, recv_row_nnz), ctypes.byref(res)), self._h)
        return res

    # ---- sharded records (multi-GPU owner routing of pair records) -------------------------------
    @staticmethod
    def shard_arena_cap(n_users: int, n_interactions: int) -> int:
        """u16 arena ids cooc_shard_plan needs for a part (a multiple of 8)."""
        return (n_interactions + 7 * max(n_users, 1) + 16 + 7) // 8 * 8

    def shard_plan(self, user_ptr, items, n_parts: int, desc, row_counts, arena, stream=None):
        """This part's users -> desc (int64 device [n_interactions]), row_counts (int32 device
        [n_items], owner-major), arena (int16 device [>= shard_arena_cap]).  Returns (descriptors per
        owner (np.int64 [n_parts]), arena ids used, this part's ordered pairs)."""
        send = np.zeros(n_parts, np.int64)
        info = np.zeros(2, np.int64)
        n_users = int(user_ptr.numel()) - 1
        check(_lib.load().cooc_shard_plan(
            self._h, n_users, ctypes.c_void_p(user_ptr.data_ptr()), ctypes.c_void_p(items.data_ptr()),
            int(items.numel()), n_parts, ctypes.c_void_p(desc.data_ptr()) if desc.numel() else None,
            ctypes.c_void_p(row_counts.data_ptr()), ctypes.c_void_p(arena.data_ptr()), int(arena.numel()),
            _stream_arg(stream, items), _p(send, i64p), _p(info, i64p)), self._h)
        return send, int(info[0]), int(info[1])

    def shard_count(self, n_parts: int, part: int, recv_row_counts, recv_desc, arena_all, arena_stride: int,
                    stream=None) -> CoocDeviceResult:
        """Owner `part`: complete rows part + r * n_parts from every source's records."""
        res = CoocDeviceResult()
        check(_lib.load().cooc_shard_count(
            self._h, n_parts, part, ctypes.c_void_p(recv_row_counts.data_ptr()),
            ctypes.c_void_p(recv_desc.data_ptr()) if recv_desc.numel() else None, int(recv_desc.numel()),
            ctypes.c_void_p(arena_all.data_ptr()), int(arena_stride),
            _stream_arg(stream, recv_row_counts), ctypes.byref(res)), self._h)
        return res

    def verify_batch(self, symmetry: bool = False, row_checksum=None, stream=None) -> dict:
        """cooc_verify_batch over the last count_device result: the reference's DEVELOPMENT_MODE row-sum
        check (ItemRowRescorer...java:183-193) and the CSR contract's checks, on the device.
        row_checksum: optional uint64-sized device tensor [n_items] (torch.int64 is fine) that receives
        every row's fingerprint (sum of splitmix64(col << 32 ^ count); oracle.row_checksums restates it)."""
        out = np.zeros(8, np.int64)
        flags = _lib.COOC_VERIFY_SYMMETRY if symmetry else 0
        cs = ctypes.c_void_p(row_checksum.data_ptr()) if row_checksum is not None else None
        check(_lib.load().cooc_verify_batch(self._h, flags, cs, _p(out, i64p), self._stream(stream)), self._h)
        return {"sum_counts": int(out[0]), "sum_rowsums": int(out[1]), "entries": int(out[2]),
                "rows_bad_sum": int(out[3]), "rows_bad_entries": int(out[4]),
                "asymmetric_entries": None if out[5] < 0 else int(out[5])}

    def _stream(self, stream):
        """An explicit stream as given; else torch's current stream on this context's device (the null
        stream without a GPU)."""
        if stream is not None:
            return ctypes.c_void_p(int(stream))
        try:
            import torch

            if torch.cuda.is_available():
                dev = self.device if self.device >= 0 else torch.cuda.current_device()
                return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        except ImportError:
            pass
        return None

    # ---- communicator: the RCCL sharding layer inside the library -------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        """cooc_comm_unique_id: rank 0's communicator id (128 opaque bytes) for cooc_comm_init."""
        buf = (ctypes.c_uint8 * _lib.COOC_COMM_ID_BYTES)()
        check(_lib.load().cooc_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)), None)
        return bytes(buf)

    def comm_init(self, unique_id: bytes, rank: int, world: int) -> None:
        """Join the RCCL communicator `unique_id` as `rank` of `world` (one context per GPU process)."""
        buf = (ctypes.c_uint8 * _lib.COOC_COMM_ID_BYTES).from_buffer_copy(unique_id)
        check(_lib.load().cooc_comm_init(self._h, ctypes.cast(buf, ctypes.c_void_p), int(rank), int(world)), self._h)
        self.comm_world = int(world)

    def comm_init_ops(self, rank: int, world: int, ops: CoocCommOps) -> None:
        """The library's exchange over caller collectives (cooc_comm_ops); `ops` must stay alive as long
        as the context (the context keeps a reference)."""
        check(_lib.load().cooc_comm_init_ops(self._h, int(rank), int(world), ctypes.byref(ops), None), self._h)
        self._comm_ops = ops
        self.comm_world = int(world)

    def count_owned_host(self, user_ptr, items):
        """cooc_count_owned_host: count_owned from host arrays (a JVM subtask's buffered shard); the owned
        rows become this context's batch result.  Returns (BatchResult of the owned rows, CoocOwnedInfo)."""
        up = np.ascontiguousarray(user_ptr, np.int64)
        it = np.ascontiguousarray(items, np.int32)
        info, winfo = CoocOwnedInfo(), CoocWindowInfo()
        L = _lib.load()
        check(L.cooc_count_owned_host(self._h, len(up) - 1, _p(up, i64p), _p(it, i32p), ctypes.byref(info),
                                      ctypes.byref(winfo)), self._h)
        return self.copy_batch(winfo.nnz, winfo.observed), info

    def count_owned_host_info(self, user_ptr, items):
        """cooc_count_owned_host without copying the owned rows out: (CoocWindowInfo, CoocOwnedInfo); the rows
        then stream out with copy_batch_row_ptr / copy_batch_range (what the JVM operators do)."""
        up = np.ascontiguousarray(user_ptr, np.int64)
        it = np.ascontiguousarray(items, np.int32)
        info, winfo = CoocOwnedInfo(), CoocWindowInfo()
        check(_lib.load().cooc_count_owned_host(self._h, len(up) - 1, _p(up, i64p), _p(it, i32p), ctypes.byref(info),
                                                ctypes.byref(winfo)), self._h)
        return winfo, info

    def copy_batch_row_ptr(self):
        """(row_ptr int64[M + 1], rowsum int64[M], rowsum32 int32[M]) of the last batch (cooc_copy_batch with
        the entry arrays NULL)."""
        M = self.n_items
        rp, rs, rs32 = np.zeros(M + 1, np.int64), np.zeros(M, np.int64), np.zeros(M, np.int32)
        check(_lib.load().cooc_copy_batch(self._h, _p(rp, i64p), None, None, None, _p(rs, i64p), _p(rs32, i32p)),
              self._h)
        return rp, rs, rs32

    def copy_batch_range(self, r0: int, r1: int, cap: int):
        """cooc_copy_batch_range: (cols int32, cnt uint32, cnt16 int16) of rows [r0, r1), at most cap entries."""
        cols, cnt, cnt16 = np.zeros(cap, np.int32), np.zeros(cap, np.uint32), np.zeros(cap, np.int16)
        check(_lib.load().cooc_copy_batch_range(self._h, int(r0), int(r1), int(cap), _p(cols, i32p), _p(cnt, u32p),
                                                _p(cnt16, i16p)), self._h)
        return cols, cnt, cnt16

    def topk_owned_host(self, topk: int, exact_scores: bool = False) -> None:
        """cooc_topk_owned_host: the owned rows' heaps into the context's buffers (copy_topk_range reads them)."""
        check(_lib.load().cooc_topk_owned_host(self._h, int(topk), _lib.COOC_FLAG_EXACT_SCORES if exact_scores else 0),
              self._h)

    def copy_topk_range(self, r0: int, r1: int, topk: int):
        """cooc_copy_topk_batch_range: (sizes [n], values [n, k], scores [n, k]) of rows [r0, r1)."""
        n = int(r1) - int(r0)
        sizes, vals, scores = np.zeros(n, np.int32), np.zeros((n, topk), np.int32), np.zeros((n, topk), np.float64)
        check(_lib.load().cooc_copy_topk_batch_range(self._h, int(r0), int(r1), int(topk), _p(sizes, i32p),
                                                     _p(vals, i32p), _p(scores, f64p)), self._h)
        return sizes, vals, scores

    def comm_allgather_i64(self, value: int) -> np.ndarray:
        """cooc_comm_allgather_i64: every rank's value, in rank order."""
        out = np.zeros(self.comm_world, np.int64)
        check(_lib.load().cooc_comm_allgather_i64(self._h, int(value), _p(out, i64p)), self._h)
        return out

    def count_owned(self, user_ptr, items, stream=None):
        """cooc_count_owned: this rank's users -> the rows it owns over the whole job's users (item
        counts all-reduced, owner map, histories all-gathered, owned rows counted, pairs all-reduced),
        all inside the library.  Returns (CoocDeviceResult, CoocOwnedInfo)."""
        res, info = CoocDeviceResult(), CoocOwnedInfo()
        n_users = int(user_ptr.numel()) - 1
        check(_lib.load().cooc_count_owned(self._h, n_users, ctypes.c_void_p(user_ptr.data_ptr()),
                                           ctypes.c_void_p(items.data_ptr()) if items.numel() else None,
                                           int(items.numel()), _stream_arg(stream, user_ptr), ctypes.byref(info),
                                           ctypes.byref(res)), self._h)
        return res, info

    def topk_owned(self, topk: int, sizes, values, scores, rowsum_global=None, exact_scores: bool = False,
                   stream=None) -> None:
        """cooc_topk_owned: the owned rows' row sums all-reduced, then their LLR top-k into device tensors."""
        check(_lib.load().cooc_topk_owned(
            self._h, int(topk), _lib.COOC_FLAG_EXACT_SCORES if exact_scores else 0, ctypes.c_void_p(sizes.data_ptr()),
            ctypes.c_void_p(values.data_ptr()), ctypes.c_void_p(scores.data_ptr()),
            None if rowsum_global is None else ctypes.c_void_p(rowsum_global.data_ptr()), _stream_arg(stream, sizes)),
            self._h)

    @staticmethod
    def snake_owner(counts, world: int, head: int = 4096) -> np.ndarray:
        """cooc_snake_owner (host): the owner map cooc_count_owned builds, from host item counts."""
        c = np.ascontiguousarray(counts, np.int64)
        out = np.zeros(len(c), np.int32)
        check(_lib.load().cooc_snake_owner(_p(c, i64p), len(c), int(world), int(head), _p(out, i32p)), None)
        return out

    def set_kernel_timing(self, enable: bool = True) -> None:
        check(_lib.load().cooc_set_kernel_timing(self._h, 1 if enable else 0), self._h)

    def last_sort_rows(self) -> tuple:
        """(rows, ordered pairs) the last large-universe count sent through the sort + segmented-reduce
        path (rows whose LDS hash table overflowed, or every whole row with planner="sort")."""
        rows, pairs = ctypes.c_int64(), ctypes.c_int64()
        check(_lib.load().cooc_last_sort_rows(self._h, ctypes.byref(rows), ctypes.byref(pairs)), self._h)
        return rows.value, pairs.value

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_float()
        check(_lib.load().cooc_last_kernel_ms(self._h, ctypes.byref(ms)), self._h)
        return ms.value

    # ---- streaming windows ----------------------------------------------------------------------
    def submit_batch(self, window_ts: int, user_ids, user_ptr, items) -> None:
        uid = np.ascontiguousarray(user_ids, np.int32)
        up = np.ascontiguousarray(user_ptr, np.int64)
        it = np.ascontiguousarray(items, np.int32)
        check(_lib.load().cooc_submit_batch(self._h, window_ts, len(uid), _p(uid, i32p), _p(up, i64p),
                                            _p(it, i32p)), self._h)

    def finish_window(self, window_ts: int) -> WindowResult:
        return self._window(self.finish_window_info(window_ts))

    def finish_window_info(self, window_ts: int) -> CoocWindowInfo:
        """Process the staged window; its outputs stay on the device until window_result()."""
        info = CoocWindowInfo()
        check(_lib.load().cooc_finish_window(self._h, window_ts, ctypes.byref(info)), self._h)
        return info

    def window_result(self, info: CoocWindowInfo) -> WindowResult:
        return self._window(info)

    def _window(self, info: CoocWindowInfo) -> WindowResult:
        L = _lib.load()
        R, nnz = info.n_rows, info.nnz
        rows = np.zeros(R, np.int32)
        rp = np.zeros(R + 1, np.int64)
        cols = np.zeros(nnz, np.int32)
        cnt = np.zeros(nnz, np.uint32)
        cnt16 = np.zeros(nnz, np.int16)
        check(L.cooc_copy_window_delta(self._h, _p(rows, i32p), _p(rp, i64p), _p(cols, i32p), _p(cnt, u32p),
                                       _p(cnt16, i16p)), self._h)
        rs_items = np.zeros(R, np.int32)
        rs = np.zeros(R, np.int64)
        rs32 = np.zeros(R, np.int32)
        check(L.cooc_copy_window_rowsums(self._h, _p(rs_items, i32p), _p(rs, i64p), _p(rs32, i32p)), self._h)
        w = WindowResult(info.ts, rows, rp, cols, cnt.astype(np.int64), cnt16, rs_items, rs, rs32, info.observed)
        if info.topk > 0:
            k = info.topk
            tr = np.zeros(info.n_topk, np.int32)
            ts = np.zeros(info.n_topk, np.int32)
            tv = np.zeros((info.n_topk, k), np.int32)
            tsc = np.zeros((info.n_topk, k), np.float64)
            if info.n_topk:
                check(L.cooc_copy_window_topk(self._h, _p(tr, i32p), _p(ts, i32p), _p(tv, i32p), _p(tsc, f64p)),
                      self._h)
            w.topk_rows, w.topk_sizes, w.topk_values, w.topk_scores = tr, ts, tv, tsc
        return w

    def global_rowsums(self):
        M = self.n_items
        ex = np.zeros(M, np.int64)
        v32 = np.zeros(M, np.int32)
        check(_lib.load().cooc_global_rowsums(self._h, _p(ex, i64p), _p(v32, i32p)), self._h)
        return ex, v32

    def global_observed(self):
        ex = ctypes.c_int64()
        ref = ctypes.c_int64()
        check(_lib.load().cooc_global_observed(self._h, ctypes.byref(ex), ctypes.byref(ref)), self._h)
        return ex.value, ref.value

    def global_row(self, item: int):
        L = _lib.load()
        n = ctypes.c_int64()
        check(L.cooc_global_row_nnz(self._h, item, ctypes.byref(n)), self._h)
        cols = np.zeros(n.value, np.int32)
        cnt = np.zeros(n.value, np.uint32)
        cnt16 = np.zeros(n.value, np.int16)
        check(L.cooc_global_row(self._h, item, _p(cols, i32p), _p(cnt, u32p), _p(cnt16, i16p)), self._h)
        return cols, cnt, cnt16

    # ---- operator mirror ------------------------------------------------------------------------
    def op_process_elements(self, users, items, ts) -> int:
        u = np.ascontiguousarray(users, np.int32)
        i = np.ascontiguousarray(items, np.int32)
        t = np.ascontiguousarray(ts, np.int64)
        late = ctypes.c_int64()
        check(_lib.load().cooc_op_process_elements(self._h, len(u), _p(u, i32p), _p(i, i32p), _p(t, i64p),
                                                   ctypes.byref(late)), self._h)
        return late.value

    def op_process_watermark(self, watermark: int) -> list[WindowResult]:
        out = []
        L = _lib.load()
        while True:
            fired = ctypes.c_int32()
            info = CoocWindowInfo()
            check(L.cooc_op_process_watermark(self._h, watermark, ctypes.byref(fired), ctypes.byref(info)), self._h)
            if not fired.value:
                return out
            out.append(self._window(info))

    def op_counters(self) -> dict:
        a = np.zeros(5, np.int64)
        check(_lib.load().cooc_op_counters(self._h, _p(a, i64p)), self._h)
        return {
            "UserInteractionCounterLateElements": int(a[0]),
            "UserInteractionCounterObservedCooccurrences": int(a[1]),
            "RowSumProcessWindowRowSum": int(a[2]),
            "ItemRowRescorerRescoredItems": int(a[3]),
            "rescorer_observed": int(a[4]),
        }


class NonSampledUserInteractionCounterOneInputStreamOperator:
    """Drop-in for the `--skip-cuts` operator chain (FlinkCooccurrences.java:65-74,135-167).

    ``NonSampledUserInteractionCounterOneInputStreamOperator(windowSize, windowUnit)`` plus the
    rescorer's ``topK`` (ItemRowRescorerTwoInputStreamOperator(short topK), :51-56) and the item-id
    universe the device tables are sized for.
    """

    ITEM_TAG = "itemCooccurrences"  # NonSampled...java:41-42
    ROW_SUM_TAG = "rowSums"         # NonSampled...java:45-46

    def __init__(self, window_size: int, window_unit: str = "MILLISECONDS", *, n_items: int, top_k: int = 10,
                 device: int = -1, exact_scores: bool = False, planner: str = "auto", user_cut: int = 0):
        """user_cut (kMax, 0 = off): expand only the first user_cut interactions of every user
        (UserInteractionCounter...java:168-205 without its random reservoir branch)."""
        if top_k <= 0:  # ItemRowRescorer...java:52-54
            raise _lib.IllegalArgumentException(_lib.COOC_ERR_ARG, f"{top_k} is <= 0")
        self.core = CooccurrenceCore(n_items, top_k, window_size_ms(window_size, window_unit), device, exact_scores,
                                     planner=planner, user_cut=user_cut)

    def process_element(self, user: int, item: int, timestamp: int) -> bool:
        """Returns True when the record was late and dropped (NonSampled...java:89-91)."""
        return self.core.op_process_elements([user], [item], [timestamp]) == 1

    def process_elements(self, users, items, timestamps) -> int:
        return self.core.op_process_elements(users, items, timestamps)

    def process_watermark(self, watermark: int) -> list[WindowResult]:
        return self.core.op_process_watermark(watermark)

    def accumulators(self) -> dict:
        return self.core.op_counters()

    def close(self):
        self.core.close()


# ---- ItemCooccurrences wire codec (ItemCooccurrences.java:113-147) --------------------------------
def encode_item_cooccurrences(items, increments, rec_ptr, others, ks=None) -> bytes:
    """Records (item, increment, others[rec_ptr[r]:rec_ptr[r+1]]) in the Kryo wire format of
    ItemCooccurrences.Serializer.write; ks[r] != -1 skips slot k of record r (:124-131)."""
    it = np.ascontiguousarray(items, np.int32)
    inc = np.ascontiguousarray(increments, np.int16)
    rp = np.ascontiguousarray(rec_ptr, np.int64)
    ot = np.ascontiguousarray(others, np.int32)
    kk = None if ks is None else np.ascontiguousarray(ks, np.int32)
    L = _lib.load()
    n = ctypes.c_int64()
    args = (len(it), _p(it, i32p), _p(inc, i16p), None if kk is None else _p(kk, i32p), _p(rp, i64p), _p(ot, i32p))
    check(L.cooc_records_encode(*args, None, 0, ctypes.byref(n)), None)
    out = np.zeros(max(n.value, 1), np.uint8)
    check(L.cooc_records_encode(*args, out.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n)), None)
    return out[: n.value].tobytes()


def decode_item_cooccurrences(data: bytes):
    """ItemCooccurrences.Serializer.read over a byte stream of records -> (items int32,
    increments int16, rec_ptr int64, others int32)."""
    buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
    L = _lib.load()
    nr, no = ctypes.c_int64(), ctypes.c_int64()
    bp = buf.ctypes.data_as(ctypes.c_void_p)
    check(L.cooc_records_decode(bp, len(data), ctypes.byref(nr), ctypes.byref(no), None, None, None, None), None)
    items = np.zeros(nr.value, np.int32)
    inc = np.zeros(nr.value, np.int16)
    rp = np.zeros(nr.value + 1, np.int64)
    ot = np.zeros(no.value, np.int32)
    check(L.cooc_records_decode(bp, len(data), ctypes.byref(nr), ctypes.byref(no), _p(items, i32p), _p(inc, i16p),
                                _p(rp, i64p), _p(ot, i32p)), None)
    return items, inc, rp, ot


# ---- text ingest (FlinkCooccurrences.java:55-61,207-229) -------------------------------------------
def parse_interactions(data: bytes):
    """'\\n'-delimited "user,item,timestamp" lines -> (users int32, items int32, ts int64), with the
    reference's InteractionLineSplitter semantics; a rejected line raises IllegalArgumentException
    naming its 0-based index."""
    L = _lib.load()
    n, bad = ctypes.c_int64(), ctypes.c_int64()
    check(L.cooc_parse_interactions(data, len(data), 0, None, None, None, ctypes.byref(n), ctypes.byref(bad)), None)
    users = np.zeros(n.value, np.int32)
    items = np.zeros(n.value, np.int32)
    ts = np.zeros(n.value, np.int64)
    st = L.cooc_parse_interactions(data, len(data), n.value, _p(users, i32p), _p(items, i32p), _p(ts, i64p),
                                   ctypes.byref(n), ctypes.byref(bad))
    if st != _lib.COOC_OK:
        raise _lib.IllegalArgumentException(st, f"line {bad.value} is not 'user,item,timestamp'")
    return users, items, ts


def run_text_source(op, data: bytes, records_per_watermark: int = 100_000) -> list:
    """Drive an operator from the job's text input: records in file order, and after every
    records_per_watermark records the AscendingTimestampExtractor watermark (largest timestamp so far
    - 1, FlinkCooccurrences.java:221-229); Long.MAX_VALUE at the end of the input (PROCESS_ONCE)."""
    users, items, ts = parse_interactions(data)
    out, hi = [], None
    for lo in range(0, len(users), records_per_watermark):
        sl = slice(lo, lo + records_per_watermark)
        op.process_elements(users[sl], items[sl], ts[sl])
        m = int(ts[sl].max())
        hi = m if hi is None else max(hi, m)
        out += op.process_watermark(hi - 1)
    out += op.process_watermark(2**63 - 1)
    return out
