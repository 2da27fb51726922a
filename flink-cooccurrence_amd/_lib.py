"""ctypes binding of include/cooc.h (the C-ABI of libcooc_hip.so).

This is the Python counterpart of the JNI/Panama stubs in INTEGRATION.md: same entry points,
same two-phase copy protocol.  Loading fails loudly when the HIP library is missing — the product
path has no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# COOC_LIB: another build of the library (A/B runs of kernel variants built next to the release one)
LIB_PATH = os.environ.get("COOC_LIB") or os.path.join(HERE, "csrc", "libcooc_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "cooc.h")

COOC_OK = 0
COOC_ERR_ARG = 1
COOC_ERR_STATE = 2
COOC_ERR_HIP = 3
COOC_ERR_OOM = 4
COOC_ERR_OVERFLOW = 5
COOC_FLAG_EXACT_SCORES = 1
COOC_FLAG_OUTPUT_CSR = 2
COOC_FLAG_OUTPUT_DENSE = 4
COOC_FLAG_GENERAL_PLANNER = 8
COOC_FLAG_SORT_ROWS = 16
COOC_FLAG_COLUMN_ORDER = 32
COOC_FLAG_ANY_ORDER = 64
COOC_VERIFY_SYMMETRY = 1

i16p = ctypes.POINTER(ctypes.c_int16)
i32p = ctypes.POINTER(ctypes.c_int32)
u32p = ctypes.POINTER(ctypes.c_uint32)
i64p = ctypes.POINTER(ctypes.c_int64)
f64p = ctypes.POINTER(ctypes.c_double)
vp = ctypes.c_void_p


class CoocConfig(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("n_items", ctypes.c_int32),
        ("topk", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("window_size_ms", ctypes.c_int64),
        ("user_cut", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class CoocWindowInfo(ctypes.Structure):
    _fields_ = [
        ("ts", ctypes.c_int64),
        ("nnz", ctypes.c_int64),
        ("observed", ctypes.c_int64),
        ("n_rows", ctypes.c_int32),
        ("topk", ctypes.c_int32),
        ("n_topk", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class CoocDeviceResult(ctypes.Structure):
    _fields_ = [
        ("n_items", ctypes.c_int64),
        ("nnz", ctypes.c_int64),
        ("observed", ctypes.c_int64),
        ("row_base", vp),
        ("row_nnz", vp),
        ("col", vp),
        ("cnt", vp),
        ("rowsum", vp),
        ("dense", vp),
    ]


class CoocOwnedInfo(ctypes.Structure):
    _fields_ = [
        ("part", ctypes.c_int32),
        ("n_parts", ctypes.c_int32),
        ("observed", ctypes.c_int64),
        ("local_observed", ctypes.c_int64),
        ("n_users_all", ctypes.c_int64),
        ("n_interactions_all", ctypes.c_int64),
        ("gathered_bytes", ctypes.c_int64),
        ("owner", vp),
        ("item_counts", vp),
    ]


# cooc_comm_ops: caller collectives (include/cooc.h)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, vp, vp, ctypes.c_int64, vp)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, vp, vp, vp, ctypes.c_int64, vp)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, vp, vp, i64p, i64p, vp, i64p, i64p, vp)


class CoocCommOps(ctypes.Structure):
    _fields_ = [("allreduce_sum_i64", ALLREDUCE_FN), ("allgather", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN)]


COOC_COMM_ID_BYTES = 128

_SIGS = {
    "cooc_abi_version": (ctypes.c_int, []),
    "cooc_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "cooc_create": (ctypes.c_int, [ctypes.POINTER(CoocConfig), ctypes.POINTER(vp)]),
    "cooc_create_on": (ctypes.c_int, [ctypes.POINTER(CoocConfig), i32p, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.POINTER(vp)]),
    "cooc_destroy": (None, [vp]),
    "cooc_last_error": (ctypes.c_char_p, [vp]),
    "cooc_count_device": (ctypes.c_int, [vp, ctypes.c_int64, vp, vp, ctypes.c_int64, vp,
                                         ctypes.POINTER(CoocDeviceResult)]),
    "cooc_item_counts": (ctypes.c_int, [vp, vp, ctypes.c_int64, vp, vp]),
    "cooc_count_device_owned": (ctypes.c_int, [vp, ctypes.c_int64, vp, vp, ctypes.c_int64, vp, ctypes.c_int32, vp,
                                               ctypes.c_int64, vp, ctypes.POINTER(CoocDeviceResult)]),
    "cooc_copy_column_order": (ctypes.c_int, [vp, i32p]),
    "cooc_count_host": (ctypes.c_int, [vp, ctypes.c_int64, i64p, i32p, ctypes.POINTER(CoocWindowInfo)]),
    "cooc_copy_batch": (ctypes.c_int, [vp, i64p, i32p, u32p, i16p, i64p, i32p]),
    "cooc_copy_batch_range": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, i32p, u32p, i16p]),
    "cooc_topk_batch": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, vp]),
    "cooc_copy_topk_batch": (ctypes.c_int, [vp, i32p, i32p, f64p]),
    "cooc_topk_batch_device": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp]),
    "cooc_llr": (ctypes.c_int, [vp, ctypes.c_int64, i64p, f64p]),
    "cooc_topk_items": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, i32p, i32p, i32p, f64p]),
    "cooc_submit_batch": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.c_int32, i32p, i64p, i32p]),
    "cooc_finish_window": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.POINTER(CoocWindowInfo)]),
    "cooc_copy_window_delta": (ctypes.c_int, [vp, i32p, i64p, i32p, u32p, i16p]),
    "cooc_copy_window_delta_range": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, i32p, u32p,
                                                    i16p]),
    "cooc_copy_window_rowsums": (ctypes.c_int, [vp, i32p, i64p, i32p]),
    "cooc_copy_window_topk": (ctypes.c_int, [vp, i32p, i32p, i32p, f64p]),
    "cooc_global_rowsums": (ctypes.c_int, [vp, i64p, i32p]),
    "cooc_global_observed": (ctypes.c_int, [vp, i64p, i64p]),
    "cooc_global_row_nnz": (ctypes.c_int, [vp, ctypes.c_int32, i64p]),
    "cooc_global_row": (ctypes.c_int, [vp, ctypes.c_int32, i32p, u32p, i16p]),
    "cooc_op_process_elements": (ctypes.c_int, [vp, ctypes.c_int64, i32p, i32p, i64p, i64p]),
    "cooc_op_process_watermark": (ctypes.c_int, [vp, ctypes.c_int64, i32p, ctypes.POINTER(CoocWindowInfo)]),
    "cooc_op_counters": (ctypes.c_int, [vp, i64p]),
    "cooc_partition_plan": (ctypes.c_int, [vp, ctypes.c_int32, i64p]),
    "cooc_partition_pack": (ctypes.c_int, [vp, ctypes.c_int32, vp, vp, vp]),
    "cooc_copy_rowsum_device": (ctypes.c_int, [vp, vp, vp]),
    "cooc_merge_partitions": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp,
                                             ctypes.POINTER(CoocDeviceResult)]),
    "cooc_comm_unique_id": (ctypes.c_int, [vp]),
    "cooc_comm_init": (ctypes.c_int, [vp, vp, ctypes.c_int32, ctypes.c_int32]),
    "cooc_comm_init_ops": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(CoocCommOps), vp]),
    "cooc_count_owned": (ctypes.c_int, [vp, ctypes.c_int64, vp, vp, ctypes.c_int64, vp, ctypes.POINTER(CoocOwnedInfo),
                                        ctypes.POINTER(CoocDeviceResult)]),
    "cooc_topk_owned": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp]),
    "cooc_count_owned_host": (ctypes.c_int, [vp, ctypes.c_int64, i64p, i32p, ctypes.POINTER(CoocOwnedInfo),
                                             ctypes.POINTER(CoocWindowInfo)]),
    "cooc_topk_owned_host": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32]),
    "cooc_copy_topk_batch_range": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, i32p, i32p,
                                                  f64p]),
    "cooc_comm_allgather_i64": (ctypes.c_int, [vp, ctypes.c_int64, i64p]),
    "cooc_snake_owner": (ctypes.c_int, [i64p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, i32p]),
    "cooc_shard_plan": (ctypes.c_int, [vp, ctypes.c_int64, vp, vp, ctypes.c_int64, ctypes.c_int32, vp, vp, vp,
                                       ctypes.c_int64, vp, i64p, i64p]),
    "cooc_shard_count": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, ctypes.c_int64, vp,
                                        ctypes.c_int64, vp, ctypes.POINTER(CoocDeviceResult)]),
    "cooc_records_encode": (ctypes.c_int, [ctypes.c_int64, i32p, i16p, i32p, i64p, i32p, vp, ctypes.c_int64,
                                           i64p]),
    "cooc_records_decode": (ctypes.c_int, [vp, ctypes.c_int64, i64p, i64p, i32p, i16p, i64p, i32p]),
    "cooc_parse_interactions": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64, i32p, i32p, i64p,
                                               i64p, i64p]),
    "cooc_verify_batch": (ctypes.c_int, [vp, ctypes.c_int32, vp, i64p, vp]),
    "cooc_set_kernel_timing": (ctypes.c_int, [vp, ctypes.c_int32]),
    "cooc_last_kernel_ms": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_float)]),
    "cooc_last_sort_rows": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "cooc_selftest_scan": (ctypes.c_int, [vp, vp, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), vp]),
    "cooc_selftest_radix": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.c_int32, vp]),
    "cooc_selftest_select": (ctypes.c_int, [vp, ctypes.c_int64, vp, vp, vp]),
}

_lib = None


class HipLibraryMissing(RuntimeError):
    pass


def header_symbols() -> list[str]:
    """Every function include/cooc.h declares (the symbol contract of the library)."""
    text = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"^COOC_API\s+[\w\s\*]*?\b(cooc_\w+)\(", text, re.M)))


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HipLibraryMissing(
            f"{LIB_PATH} is missing: build it with __graft_entry__.build() (make -C flink-cooccurrence_amd/csrc). "
            "The co-occurrence core has no CPU fallback."
        )
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


class CoocError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"[{status}] {msg}")
        self.status = status


class IllegalArgumentException(CoocError, ValueError):
    pass


class IllegalStateException(CoocError):
    pass


def check(status: int, ctx=None):
    if status == COOC_OK:
        return
    L = load()
    msg = (L.cooc_last_error(ctx) or b"").decode(errors="replace")
    if not msg:
        msg = L.cooc_status_string(status).decode()
    if status == COOC_ERR_ARG:
        raise IllegalArgumentException(status, msg)
    if status == COOC_ERR_STATE:
        raise IllegalStateException(status, msg)
    raise CoocError(status, msg)
