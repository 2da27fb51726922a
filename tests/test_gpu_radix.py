"""The planner's hand-written stable LSD radix sort and flag compaction (flink-cooccurrence_amd/csrc/cooc_radix.h)
against numpy's stable sort, through cooc_selftest_radix / cooc_selftest_select: the contributions' sort by item
(u32 keys, 20 bits), the work queue's and the relabel's descending sorts of u64 keys over a partial bit range, tails
below one 4,096-key tile and across many, skewed digits (a Zipf head), equal keys (stability), full-width keys.
Needs an MI355X."""
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


def _sort(lib, torch, keys, vals, bit0, bit1, desc):
    kin = torch.from_numpy(keys).cuda()
    vin = torch.from_numpy(vals.view(np.int32)).cuda()
    kout = torch.empty_like(kin)
    vout = torch.empty_like(vin)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = lib.cooc_selftest_radix(ctypes.c_void_p(kin.data_ptr()), ctypes.c_void_p(vin.data_ptr()),
                                 ctypes.c_void_p(kout.data_ptr()), ctypes.c_void_p(vout.data_ptr()), keys.size,
                                 keys.itemsize, bit0, bit1, int(desc), stream)
    assert rc == 0, lib.cooc_last_error(None)
    got_k = kout.cpu().numpy()
    got_v = vout.cpu().numpy().view(np.uint32)
    assert np.array_equal(kin.cpu().numpy(), keys)  # the inputs stay as they were
    return got_k, got_v


def _want(keys, vals, bit0, bit1, desc):
    width = bit1 - bit0
    k = keys.astype(np.uint64)
    field = (k >> np.uint64(bit0)) & np.uint64((1 << width) - 1) if width < 64 else k
    if desc:
        field = np.uint64((1 << width) - 1 if width < 64 else 0xFFFFFFFFFFFFFFFF) - field
    perm = np.argsort(field, kind="stable")
    return keys[perm], vals[perm]


CASES = [  # (n, key bytes, bit0, bit1, descending, distribution)
    (1, 4, 0, 20, False, "uniform"),
    (100, 4, 0, 20, False, "uniform"),
    (4095, 4, 0, 20, False, "zipf"),
    (4096, 4, 0, 20, False, "zipf"),
    (4097, 4, 0, 20, False, "uniform"),
    (300_000, 4, 0, 20, False, "zipf"),
    (3_000_001, 4, 0, 20, False, "zipf"),
    (200_000, 4, 0, 32, False, "uniform"),
    (200_000, 4, 3, 17, True, "uniform"),
    (200_000, 4, 0, 20, False, "equal"),
    (1_000_000, 8, 0, 35, True, "zipf"),
    (1_000_000, 8, 0, 21, True, "uniform"),
    (123_457, 8, 0, 64, False, "uniform"),
    (123_457, 8, 0, 64, True, "uniform"),
    (65_536, 8, 30, 45, False, "zipf"),
]


@pytest.mark.parametrize("n,kb,bit0,bit1,desc,dist", CASES)
def test_radix_sort_vs_numpy_stable(pkg, torch_cuda, n, kb, bit0, bit1, desc, dist):
    torch = torch_cuda
    from flink_cooccurrence_amd import _lib

    lib = _lib.load()
    rng = np.random.default_rng(n + 7 * bit0 + 13 * bit1 + int(desc))
    dt = np.uint32 if kb == 4 else np.uint64
    top = (1 << min(bit1, 8 * kb)) - 1 if bit1 < 64 else (1 << 64) - 1
    if dist == "uniform":
        keys = rng.integers(0, top, n, dtype=np.uint64, endpoint=True).astype(dt)
    elif dist == "zipf":  # a heavy head: most keys small, repeated
        keys = np.minimum(rng.zipf(1.3, n).astype(np.uint64) - 1, np.uint64(top)).astype(dt)
        keys = (keys << np.uint64(bit0)).astype(dt) if bit0 else keys
    else:
        keys = np.full(n, 12345, dt)
    vals = np.arange(n, dtype=np.uint32)  # the input position: stability is visible in the values
    got_k, got_v = _sort(lib, torch, keys, vals, bit0, bit1, desc)
    want_k, want_v = _want(keys, vals, bit0, bit1, desc)
    assert np.array_equal(got_k, want_k), f"keys differ at {np.flatnonzero(got_k != want_k)[:3]}"
    assert np.array_equal(got_v, want_v), f"values differ (stability) at {np.flatnonzero(got_v != want_v)[:3]}"


def test_radix_sort_empty_and_bad_args(pkg, torch_cuda):
    torch = torch_cuda
    from flink_cooccurrence_amd import _lib

    lib = _lib.load()
    x = torch.zeros(4, dtype=torch.int64, device="cuda")
    assert lib.cooc_selftest_radix(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                   ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()), 0, 4, 0, 20, 0,
                                   None) == 0
    assert lib.cooc_selftest_radix(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                   ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()), 4, 2, 0, 20, 0,
                                   None) == _lib.COOC_ERR_ARG
    assert lib.cooc_selftest_radix(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                   ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()), 4, 4, 0, 33, 0,
                                   None) == _lib.COOC_ERR_ARG


@pytest.mark.parametrize("n,p", [(0, 0.5), (1, 1.0), (4095, 0.01), (4097, 0.5), (1_000_000, 0.016), (300_001, 1.0)])
def test_select_flagged_vs_numpy(pkg, torch_cuda, n, p):
    torch = torch_cuda
    from flink_cooccurrence_amd import _lib

    lib = _lib.load()
    rng = np.random.default_rng(n)
    flags = (rng.random(n) < p).astype(np.uint8)
    f = torch.from_numpy(flags).cuda() if n else torch.zeros(1, dtype=torch.uint8, device="cuda")
    out = torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda")
    n_sel = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.cooc_selftest_select(ctypes.c_void_p(f.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
                                    ctypes.c_void_p(n_sel.data_ptr()), stream) == 0
    want = np.flatnonzero(flags).astype(np.int32)
    assert int(n_sel.item()) == want.size
    assert np.array_equal(out.cpu().numpy()[: want.size], want)
