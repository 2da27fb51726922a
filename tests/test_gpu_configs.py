"""BASELINE.json's configs on the GPU at their stated sizes, plus the device LLR
against the reference's known answers.  Needs an MI355X.

- C1 (10k users x 1k items, Poisson(20), Zipf(1.0) with replacement, 1 s windows over ms timestamps):
  every fired window and the final global state against the oracle's record-by-record operator.
- C4 (the C2 log over 100 tumbling 1 s windows): size-independent checks -- the windows' observed
  pairs sum to P = sum_u n_u (n_u - 1), every window's row-sum deltas sum to its observed pairs,
  the global row sums equal the closed form sum_u m_u(a) (n_u - 1), and sampled global rows equal
  rows summed directly from the users' lists.
- LogLikelihoodTest.java:14-16 through the device function the rescoring kernels use.
"""
import numpy as np
import pytest

from tests._helpers import INT64_MAX, assert_windows_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_device_llr_known_answers(pkg, oracle, torch_cuda):
    k = np.array([[110, 2442, 111, 29114], [29, 13, 123, 31612], [9, 12, 429, 31327],  # LogLikelihoodTest.java:14-16
                  [0, 0, 0, 0], [1, 0, 0, 0], [5, 0, 0, 5],                               # clamp / xLogX(0) cases
                  [3, 7, 9, 81], [40000, 123456, 7890, 10 ** 9]], np.int64)
    with pkg.CooccurrenceCore(n_items=10, device=0) as core:
        got = core.llr(k)
    # the reference's own tolerance (0.1) on its three cases ...
    assert got[:3] == pytest.approx([270.72, 263.90, 48.94], abs=0.1)
    assert got[3] == 0.0 and got[4] == 0.0 and got[5] > 0.0
    # ... and the oracle's restatement bit for bit: the same operation order, contraction off, and the same log
    # (Java's StrictMath.log, fdlibm's __ieee754_log, on both sides)
    want = np.array([oracle.llr(*map(int, r)) for r in k])
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_device_llr_bit_exact_vs_oracle(pkg, oracle, torch_cuda):
    """200,000 contingency tables spanning the rescorer's ranges (k11 from the int16 view, row sums up to the
    int32 range, observed totals up to 3e11, negative cells from wrapped views -> NaN): the device LLR
    (LogLikelihood.java:41-57 with fdlibm's log) equals the oracle's bit for bit, NaN where NaN."""
    rng = np.random.default_rng(5)
    n = 200_000
    k11 = rng.integers(-32768, 32768, n)
    k11[: n // 2] = rng.integers(0, 64, n // 2)  # (most entries: small counts)
    rs_a = rng.integers(-(1 << 31), 1 << 31, n)
    rs_b = rng.integers(-(1 << 31), 1 << 31, n)
    rs_a[: n // 2] = np.abs(rs_a[: n // 2]) // 1024 + 64
    rs_b[: n // 2] = np.abs(rs_b[: n // 2]) // 1024 + 64
    obs = rng.integers(0, 3 * 10 ** 11, n)
    k12, k21 = rs_a - k11, rs_b - k11
    k = np.stack([k11, k12, k21, obs + k11 - k12 - k21], 1).astype(np.int64)
    with pkg.CooccurrenceCore(n_items=10, device=0) as core:
        got = core.llr(k)
    want = np.array([oracle.llr(*map(int, r)) for r in k])
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan) and nan.any() and (~nan).sum() > n // 2
    bad = np.flatnonzero(got[~nan].view(np.uint64) != want[~nan].view(np.uint64))
    assert len(bad) == 0, f"{len(bad)} scores differ, e.g. {got[~nan][bad[:3]]} vs {want[~nan][bad[:3]]}"


def test_c1_full_size_vs_oracle_stream(pkg, oracle, torch_cuda):
    from flink_cooccurrence_amd import datagen

    d = datagen.config_c1(seed=1)  # U = 10,000, M = 1,000, mean 20, 1 s windows
    users, items, ts = datagen.to_records(d["user_ptr"], d["items"], d["ts"])
    M = d["n_items"]
    op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1, "SECONDS", n_items=M, top_k=10)
    ref = oracle.OracleStream(1000, topk=10)
    got, want = [], []
    for lo in range(0, len(users), 25_000):  # periodic watermarks between chunks of the stream
        sl = slice(lo, lo + 25_000)
        op.process_elements(users[sl], items[sl], ts[sl])
        ref.process_elements(users[sl], items[sl], ts[sl])
        wm = int(ts[sl][-1]) - 1
        got += op.process_watermark(wm)
        want += ref.process_watermark(wm)
    got += op.process_watermark(INT64_MAX)
    want += ref.process_watermark(INT64_MAX)
    assert len(got) == len(want) >= 150
    for g, w in zip(got, want):
        assert_windows_equal(g, w)
    assert op.accumulators() == ref.counters()
    rows, rp, cols, exact, v16 = ref.global_rows()
    for r in range(0, len(rows), 7):
        c, n, n16 = op.core.global_row(int(rows[r]))
        assert np.array_equal(c, cols[rp[r]:rp[r + 1]])
        assert np.array_equal(n.astype(np.int64), exact[rp[r]:rp[r + 1]])
        assert np.array_equal(n16, v16[rp[r]:rp[r + 1]])
    gi, gv32, gex = ref.global_rowsums()
    ex, v32 = op.core.global_rowsums()
    assert np.array_equal(ex[gi], gex) and np.array_equal(v32[gi], gv32)
    op.close()


def _brute_row(up, it, order, sorted_items, users, a, M):
    """C[a, :] summed directly: sum over users u holding a of m_u(a) * counts(u's list), minus
    sum_u m_u(a) at column a."""
    lo, hi = np.searchsorted(sorted_items, [a, a + 1])
    us, mult = np.unique(users[order[lo:hi]], return_counts=True)
    lens = up[us + 1] - up[us]
    idx = np.repeat(up[us] - np.cumsum(np.concatenate([[0], lens[:-1]])), lens) + np.arange(lens.sum())
    row = np.rint(np.bincount(it[idx], weights=np.repeat(mult, lens).astype(np.float64), minlength=M)).astype(np.int64)
    row[a] -= int(mult.sum())
    nz = np.nonzero(row)[0]
    return nz.astype(np.int32), row[nz]


def test_c4_hundred_windows_properties(pkg, torch_cuda):
    from flink_cooccurrence_amd import datagen

    d = datagen.config_c4(seed=4)  # C2 log, 100 x 1 s windows
    up, it, M = d["user_ptr"], d["items"], d["n_items"]
    lens = np.diff(up)
    P = int(np.sum(lens * (lens - 1)))
    users, items, ts = datagen.to_records(up, it, d["ts"])
    op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1, "SECONDS", n_items=M, top_k=1)
    windows = []
    bounds = np.searchsorted(ts, np.arange(1, 101) * 1000)  # records of window w end at bounds[w]
    lo = 0
    for w, hi in enumerate(bounds):
        op.process_elements(users[lo:hi], items[lo:hi], ts[lo:hi])
        for r in op.process_watermark(w * 1000 + 999):
            windows.append((r.ts, r.observed, int(r.rs_exact.sum()), len(r.rows)))
        lo = hi
    assert lo == len(users)
    assert len(windows) == 100 and [w[0] for w in windows] == [w * 1000 + 999 for w in range(100)]
    assert sum(w[1] for w in windows) == P
    assert all(w[1] == w[2] for w in windows)  # row-sum deltas sum to the window's ordered pairs
    ex, _ = op.core.global_rowsums()
    want_rs = np.zeros(M, np.int64)
    np.add.at(want_rs, it.astype(np.int64), np.repeat(lens - 1, lens))
    assert np.array_equal(ex, want_rs)
    assert op.core.global_observed()[0] == P
    order = np.argsort(it, kind="stable")
    sorted_items = it[order].astype(np.int64)
    owners = np.repeat(np.arange(len(lens)), lens)
    rng = np.random.default_rng(4)
    for a in np.concatenate([[0, 1, 2, 17], rng.integers(0, M, 12)]):
        c, n, _ = op.core.global_row(int(a))
        wc, wn = _brute_row(up, it.astype(np.int64), order, sorted_items, owners, int(a), M)
        assert np.array_equal(c, wc) and np.array_equal(n.astype(np.int64), wn)
    op.close()
