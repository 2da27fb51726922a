"""The planner's hand-written single-pass prefix sum (flink-cooccurrence_amd/csrc/cooc_scan.h, k_scan_lookback)
against torch.cumsum, through cooc_selftest_scan: every variant the library launches (inclusive / exclusive,
vectorised / LDS-staged tiles, int64 / int32 input and output) at sizes below one 4,096-element tile, around tile
multiples, and with look-backs across more than 64 tiles.  Every prefix the large-universe planner indexes with
(pair work, arena bases, row pointers) comes out of this kernel.  Needs an MI355X."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TILE = 4096
SIZES = [1, 17, TILE - 1, TILE, TILE + 1, 3 * TILE + 5, 64 * TILE - 1, 64 * TILE, 64 * TILE + 1, 65 * TILE + 3,
         3 * 64 * TILE + 100, 300 * TILE + 7]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _scan(lib, torch, x, flags):
    out = torch.empty(x.numel(), dtype=torch.int32 if flags & 4 else torch.int64, device=x.device)
    diag = ctypes.c_int64(-1)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = lib.cooc_selftest_scan(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()), x.numel(), flags,
                                ctypes.byref(diag), stream)
    assert rc == 0, lib.cooc_last_error(None)
    assert diag.value == 0, f"scan diagnostic word {diag.value}"
    return out


@pytest.mark.parametrize("flags", list(range(16)))
def test_scan_variants_vs_cumsum(pkg, torch_cuda, flags):
    torch = torch_cuda
    from flink_cooccurrence_amd import _lib

    lib = _lib.load()
    rng = np.random.default_rng(1000 + flags)
    for n in SIZES:
        h = rng.integers(0, 100, n)  # (int32 outputs: the prefix stays below 2^31)
        x = torch.from_numpy(h.astype(np.int32 if flags & 8 else np.int64)).cuda()
        got = _scan(lib, torch, x, flags).cpu().numpy().astype(np.int64)
        inc = np.cumsum(h)
        want = inc if flags & 1 else inc - h
        assert np.array_equal(got, want), f"n={n} flags={flags}: first mismatch at {np.flatnonzero(got != want)[:1]}"


def test_scan_wide_values(pkg, torch_cuda):
    """int64 prefixes far above 2^32 (the pair-work prefix of the C3 planner reaches ~3e10), across 300 tiles."""
    torch = torch_cuda
    from flink_cooccurrence_amd import _lib

    lib = _lib.load()
    rng = np.random.default_rng(7)
    for flags in (0, 1, 2, 3):
        h = rng.integers(0, 1 << 40, 300 * TILE + 7)
        got = _scan(lib, torch, torch.from_numpy(h).cuda(), flags).cpu().numpy()
        inc = np.cumsum(h)
        assert np.array_equal(got, inc if flags & 1 else inc - h)


def test_scan_empty_and_bad_args(pkg, torch_cuda):
    torch = torch_cuda
    from flink_cooccurrence_amd import _lib

    lib = _lib.load()
    x = torch.zeros(4, dtype=torch.int64, device="cuda")
    out = torch.full((4,), 7, dtype=torch.int64, device="cuda")
    assert lib.cooc_selftest_scan(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()), 0, 0, None,
                                  None) == 0
    assert out.cpu().tolist() == [7, 7, 7, 7]  # n = 0 writes nothing
    assert lib.cooc_selftest_scan(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()), 4, 16, None,
                                  None) == _lib.COOC_ERR_ARG
