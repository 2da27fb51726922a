"""The C-ABI library on a machine without a GPU: it loads, exports exactly the header's entry
points, and every compute entry point fails loudly (no CPU fallback)."""
import ctypes
import subprocess

import pytest
import torch


def _exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln and ln.split()[-1].startswith("cooc_")}


def test_library_exports_every_header_symbol(pkg):
    from flink_cooccurrence_amd import _lib

    L = _lib.load()
    declared = set(_lib.header_symbols())
    assert len(declared) >= 20
    assert declared == _exported(_lib.LIB_PATH)
    for name in declared:
        assert hasattr(L, name)
    assert L.cooc_abi_version() == 7


def test_status_strings(pkg):
    from flink_cooccurrence_amd import _lib

    L = _lib.load()
    assert L.cooc_status_string(0) == b"ok"
    assert L.cooc_status_string(5) == b"uint32 count overflow"


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_create_fails_loudly_without_gpu(pkg):
    with pytest.raises(pkg.CoocError) as e:
        pkg.CooccurrenceCore(n_items=10)
    assert e.value.status == 3 and "no HIP device" in str(e.value)


def test_create_on_rejects_devices_it_cannot_see(pkg):
    """create(cfg{devices[]}): a device ordinal the runtime does not list is an argument error."""
    with pytest.raises(pkg.IllegalArgumentException):
        pkg.CooccurrenceCore(n_items=10, devices=[0], subtask=0)


def test_argument_errors_mirror_reference(pkg):
    from flink_cooccurrence_amd import _lib

    L = _lib.load()
    # ItemRowRescorer...java:52-54: topK <= 0 is an IllegalArgumentException
    with pytest.raises(pkg.IllegalArgumentException):
        pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1, "SECONDS", n_items=10, top_k=0)
    with pytest.raises(pkg.IllegalArgumentException):
        pkg.window_size_ms(1, "WEEKS")  # Configuration.java:176-177
    cfg = _lib.CoocConfig(-1, 0, 0, 0, 1000, 0, 0)
    h = ctypes.c_void_p()
    assert L.cooc_create(ctypes.byref(cfg), ctypes.byref(h)) == _lib.COOC_ERR_ARG
    assert b"n_items" in L.cooc_last_error(None)
    # userCut is a Java short (UserInteractionCounter...java:54): rejected before any device call
    cfg = _lib.CoocConfig(-1, 10, 0, 0, 1000, 40000, 0)
    assert L.cooc_create(ctypes.byref(cfg), ctypes.byref(h)) == _lib.COOC_ERR_ARG
    assert b"userCut" in L.cooc_last_error(None)


def test_window_units(pkg):
    assert pkg.window_size_ms(1, "SECONDS") == 1000
    assert pkg.window_size_ms(2, "minutes") == 120_000
