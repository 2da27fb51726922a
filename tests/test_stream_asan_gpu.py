"""The streaming operator's host bookkeeping (cooc_stream.cpp, cooc_ctx.cpp, cooc_capi.cpp) under
AddressSanitizer + UndefinedBehaviorSanitizer on the GPU: tests/sanitize/stream_driver.cpp linked with the
library built with host-side -fsanitize (scripts/build_asan.sh, which build() runs; kernels unsanitized -- GPU
sanitizers are not available on the pool).  Any out-of-bounds host access, leak-free-ness aside, or undefined
operation aborts the driver; it also checks the C-ABI operator's output invariants."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "sanitize", "stream_asan")


def test_stream_host_code_under_asan_ubsan():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.skip("tests/sanitize/stream_asan not built (scripts/build_asan.sh is best effort in build())")
    # detect_leaks=0: the HIP runtime keeps process-lifetime allocations; verify_asan_link_order=0: the
    # environment may preload a library ahead of the sanitizer runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([EXE], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "stream_asan ok" in r.stdout, r.stdout[-2000:]
