"""Parity of the HIP path (through the C-ABI) against the oracle.  Needs an MI355X.

Bar: bit-exact for every count, row sum, key set and wrapped view; LLR scores within the
condition-aware tolerance of SURVEY.md §8(a) (rtol 1e-6 here, tighter than the reference's own 0.1
KAT tolerance), top-k item sets equal strictly above the k-th score.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from tests._helpers import (INT64_MAX, as_int_keys, assert_windows_equal, micro_csr, micro_events, micro_logs,
                            run_events, window_rows, window_rows16)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _batch_vs_closed_form(pkg, oracle, up, it, M, layouts=("csr", "dense")):
    """Both result layouts of the batch path (padded CSR and dense matrix) against the closed form."""
    for output in layouts:
        got = _batch_layout_vs_closed_form(pkg, oracle, up, it, M, output)
    return got


def _batch_layout_vs_closed_form(pkg, oracle, up, it, M, output):
    with pkg.CooccurrenceCore(n_items=M, output=output) as core:
        got = core.count(up, it)
    rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
    assert got.observed == observed
    assert np.array_equal(got.row_ptr, rp), "row lengths / key sets differ"
    assert np.array_equal(got.cols, cols)
    assert np.array_equal(got.cnt.astype(np.int64), data)
    assert np.array_equal(got.cnt16, oracle.to_i16(data))
    assert np.array_equal(got.rowsum, rowsums)
    assert np.array_equal(got.rowsum32, oracle.to_i32(rowsums))
    return got


@pytest.mark.parametrize("seed,U,M,mean,repl", [
    (1, 500, 97, 12.0, True),
    (2, 3000, 1000, 20.0, True),      # C1 shape, scaled
    (3, 2000, 4096, 40.0, False),     # rating-log shape
    (4, 300, 40704, 60.0, True),      # just above the batch planner: the large-universe planner
    (6, 300, 40319, 60.0, True),     # the largest batch-planner row (+ pad sink + descriptors)
    (7, 5000, 2000, 150.0, False),    # long lists, many batches per chunk
])
def test_batch_random_logs(pkg, oracle, torch_cuda, seed, U, M, mean, repl):
    from flink_cooccurrence_amd import datagen

    up, it = datagen.small_log(seed, U, M, mean, replacement=repl)
    _batch_vs_closed_form(pkg, oracle, up, it, M)


def test_batch_matches_literal_expansion(pkg, oracle, torch_cuda):
    from flink_cooccurrence_amd import datagen

    up, it = datagen.small_log(5, 400, 64, 10.0)
    got = _batch_vs_closed_form(pkg, oracle, up, it, 64)
    dense, rs, obs = oracle.batch_dense(up, it, 64)
    C = sp.csr_matrix((got.cnt.astype(np.int64), got.cols, got.row_ptr), shape=(64, 64)).toarray()
    assert np.array_equal(C, dense) and np.array_equal(got.rowsum, rs) and got.observed == obs


@pytest.mark.parametrize("case", ["empty", "empty_users", "singletons", "one_item_universe", "max_id", "one_user",
                                  "long_lists"])
def test_batch_edge_cases(pkg, oracle, torch_cuda, case):
    M = 50
    if case == "empty":
        up, it = np.zeros(1, np.int64), np.zeros(0, np.int32)
    elif case == "empty_users":
        up, it = np.array([0, 0, 3, 3, 5, 5], np.int64), np.array([1, 2, 3, 4, 4], np.int32)
    elif case == "singletons":
        up, it = np.arange(11, dtype=np.int64), np.arange(10, dtype=np.int32)
    elif case == "one_item_universe":
        M = 1
        up, it = np.array([0, 3, 4, 8], np.int64), np.zeros(8, np.int32)
    elif case == "max_id":
        up, it = np.array([0, 4], np.int64), np.array([M - 1, 0, M - 1, 7], np.int32)
    elif case == "long_lists":  # lists beyond one planner thread (2048), between short ones
        rng = np.random.default_rng(11)
        lens = np.array([5, 3000, 0, 2049, 7, 9000, 1], np.int64)
        up = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        it = rng.integers(0, M, int(up[-1])).astype(np.int32)
    else:
        up, it = np.array([0, 30], np.int64), np.arange(30, dtype=np.int32) % 7
    _batch_vs_closed_form(pkg, oracle, up, it, M)


def test_batch_split_heavy_rows(pkg, oracle, torch_cuda):
    """Rows whose pair work exceeds one chunk (2^22) are split over workgroups and merged."""
    rng = np.random.default_rng(9)
    U, L, M = 2600, 1700, 5000
    it = np.concatenate([np.concatenate([[0, 1], rng.choice(np.arange(2, M), L - 2, replace=False)])
                         for _ in range(U)]).astype(np.int32)
    up = (np.arange(U + 1) * L).astype(np.int64)
    got = _batch_vs_closed_form(pkg, oracle, up, it, M)
    assert got.rowsum[0] == U * (L - 1) > (1 << 22)


@pytest.mark.parametrize("log", micro_logs(), ids=lambda l: l["name"])
def test_micro_logs_batch(pkg, oracle, torch_cuda, log):
    if len(log["windows"]) != 1:
        pytest.skip("multi-window log: covered by the streaming test")
    up, it = micro_csr(log)
    M = int(it.max()) + 1
    got = _batch_vs_closed_form(pkg, oracle, up, it, M)
    w = log["windows"][0]
    rows = {a: dict(zip(got.cols[got.row_ptr[a]:got.row_ptr[a + 1]].tolist(),
                        got.cnt[got.row_ptr[a]:got.row_ptr[a + 1]].astype(np.int64).tolist()))
            for a in range(M) if got.row_ptr[a + 1] > got.row_ptr[a]}
    assert rows == as_int_keys(w["rows"])
    if "rows16" in w:
        r16 = {a: dict(zip(got.cols[got.row_ptr[a]:got.row_ptr[a + 1]].tolist(),
                           got.cnt16[got.row_ptr[a]:got.row_ptr[a + 1]].tolist()))
               for a in range(M) if got.row_ptr[a + 1] > got.row_ptr[a]}
        assert r16 == as_int_keys(w["rows16"])
    if "rowsums32" in w:
        for a, v in as_int_keys(w["rowsums32"]).items():
            assert got.rowsum32[a] == v
    assert got.observed == w["observed"]


@pytest.mark.parametrize("planner", ["auto", "large", "sort"])
@pytest.mark.parametrize("log", [l for l in micro_logs() if not l.get("closed_form_only")], ids=lambda l: l["name"])
def test_micro_logs_operator(pkg, oracle, torch_cuda, log, planner):
    """The operator mirror (processElement / watermark firing / late drop) on the micro-logs, through
    the batch planner (streaming windows over resident histories), the large-universe planner (per-row LDS
    hash / dense-tile chunks) and its sort + segmented-reduce path (planner="sort")."""
    ev = micro_events(log)
    M = 1 + max(e[2] for e in ev if e[0] == "e")
    op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(log["window_ms"], n_items=M, top_k=3,
                                                                    planner=planner)
    got = run_events(ev, op.process_elements, op.process_watermark)
    ref = oracle.OracleStream(log["window_ms"], topk=3)
    want = run_events(ev, ref.process_elements, ref.process_watermark)
    assert len(got) == len(want) == len(log["windows"])
    for g, w, gold in zip(got, want, log["windows"]):
        assert_windows_equal(g, w)
        assert window_rows(g) == as_int_keys(gold["rows"])
        if "rows16" in gold:
            assert window_rows16(g) == as_int_keys(gold["rows16"])
    acc, racc = op.accumulators(), ref.counters()
    assert acc == racc
    op.close()


def test_bad_item_id_is_illegal_argument(pkg, torch_cuda):
    with pkg.CooccurrenceCore(n_items=10) as core:
        with pytest.raises(pkg.IllegalArgumentException):
            core.count(np.array([0, 2], np.int64), np.array([3, 10], np.int32))
        # the context stays usable
        got = core.count(np.array([0, 2], np.int64), np.array([3, 4], np.int32))
        assert got.observed == 2


def test_dense_view_on_a_reused_context(pkg, oracle, torch_cuda):
    """The dense device view: rows of items absent from a later batch read as zero although the
    context's matrix held counts from an earlier batch; split rows are summed across chunks."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    M = 600
    dev = torch.device("cuda")
    up1, it1 = datagen.small_log(23, 2000, M, 30.0)
    rng = np.random.default_rng(24)
    U2, L2 = 2600, 1700   # rows 0 and 1 carry U2 * (L2 - 1) > 2^22 pairs: split over chunks
    it2 = np.concatenate([np.concatenate([[0, 1], rng.choice(np.arange(2, M // 2), L2 - 2, replace=True)])
                          for _ in range(U2)]).astype(np.int32)
    up2 = (np.arange(U2 + 1) * L2).astype(np.int64)
    with pkg.CooccurrenceCore(n_items=M, device=0, output="dense") as core:
        for up, it in [(up1, it1), (up2, it2)]:
            res = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
            torch.cuda.synchronize()
            assert res.dense and not res.col and not res.row_base
            D = _d2h(res.dense, M * M, np.uint32).reshape(M, M).astype(np.int64)
            rp, cols, data, rs, obs = oracle.closed_form(up, it, M)
            want = sp.csr_matrix((data, cols, rp), shape=(M, M)).toarray()
            assert np.array_equal(D, want) and res.observed == obs
            assert np.array_equal(_d2h(res.row_nnz, M, np.int32), (want != 0).sum(1))
            assert np.array_equal(_d2h(res.rowsum, M, np.int64), rs)
            assert res.nnz == int((want != 0).sum())


def test_count_device_padded_layout(pkg, oracle, torch_cuda):
    import ctypes

    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    up, it = datagen.small_log(21, 1000, 300, 15.0)
    dev = torch.device("cuda")
    with pkg.CooccurrenceCore(n_items=300, device=0, output="csr") as core:
        core.set_kernel_timing(True)
        res = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
        assert core.last_kernel_ms() > 0
        rp, cols, data, rowsums, observed = oracle.closed_form(up, it, 300)
        assert res.observed == observed and res.nnz == len(cols)
        got = core.copy_batch(res.nnz, res.observed)
        assert np.array_equal(got.cols, cols)
        # borrowed device views: row_nnz matches the packed row lengths
        nnz = np.zeros(300, np.int32)
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy(nnz.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(res.row_nnz), ctypes.c_size_t(1200),
                      ctypes.c_int(2))
        assert np.array_equal(nnz, np.diff(rp))


@pytest.mark.parametrize("planner", ["auto", "large", "sort"])
def test_streaming_windows_vs_oracle(pkg, oracle, torch_cuda, planner):
    """C1-shaped click log over 1 s windows: every window's delta rows, row sums, observed, the
    rescorer's top-k, and the final global state."""
    from flink_cooccurrence_amd import datagen

    d = datagen.config_c1(seed=1, U=2000, M=300, mean=20.0)
    users, items, ts = datagen.to_records(d["user_ptr"], d["items"], d["ts"])
    op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1, "SECONDS", n_items=300, top_k=10,
                                                                    planner=planner)
    ref = oracle.OracleStream(1000, topk=10)
    got, want = [], []
    for lo in range(0, len(users), 7000):  # watermarks between chunks, like periodic watermarks
        sl = slice(lo, lo + 7000)
        op.process_elements(users[sl], items[sl], ts[sl])
        ref.process_elements(users[sl], items[sl], ts[sl])
        wm = int(ts[sl][-1]) - 1
        got += op.process_watermark(wm)
        want += ref.process_watermark(wm)
    got += op.process_watermark(INT64_MAX)
    want += ref.process_watermark(INT64_MAX)
    assert len(got) == len(want) > 10
    for g, w in zip(got, want):
        assert_windows_equal(g, w)
    assert op.accumulators() == ref.counters()
    rows, rp, cols, exact, v16 = ref.global_rows()
    for r, a in enumerate(rows[:50]):
        c, n, n16 = op.core.global_row(int(a))
        assert np.array_equal(c, cols[rp[r]:rp[r + 1]])
        assert np.array_equal(n.astype(np.int64), exact[rp[r]:rp[r + 1]])
        assert np.array_equal(n16, v16[rp[r]:rp[r + 1]])
    gi, gv32, gex = ref.global_rowsums()
    ex, v32 = op.core.global_rowsums()
    assert np.array_equal(ex[gi], gex) and np.array_equal(v32[gi], gv32)
    op.close()


@pytest.mark.parametrize("planner", ["auto", "large", "sort"])
def test_streaming_long_histories_vs_closed_form(pkg, oracle, torch_cuda, planner):
    """Windows over resident histories longer than one fill thread's share (2,048 ids), with
    repeats, users absent from some windows, and a row (item 0) split over several chunks: every
    window's delta rows, row sums and observed equal the closed-form difference
    C(A through window w) - C(A through window w - 1)."""
    rng = np.random.default_rng(31)
    M, n_win = 500, 3
    heavy = [np.where(rng.random(3000) < 0.1, 0, rng.integers(1, M, 3000)) for _ in range(40)]
    light = [rng.integers(0, M, int(rng.integers(1, 40))) for _ in range(2000)]
    lists = heavy + light
    parts = [[l[len(l) * w // n_win:len(l) * (w + 1) // n_win] for l in lists] for w in range(n_win)]
    C_prev = sp.csr_matrix((M, M), dtype=np.int64)
    rs_prev, obs_prev = np.zeros(M, np.int64), 0
    with pkg.CooccurrenceCore(n_items=M, planner=planner) as core:
        for w in range(n_win):
            uids = [u for u in range(len(lists)) if len(parts[w][u])]
            up = np.concatenate([[0], np.cumsum([len(parts[w][u]) for u in uids])]).astype(np.int64)
            it = np.concatenate([parts[w][u] for u in uids]).astype(np.int32)
            core.submit_batch(w * 1000 + 999, np.array(uids, np.int32), up, it)
            got = core.finish_window(w * 1000 + 999)
            cum = [np.concatenate([parts[v][u] for v in range(w + 1)]) for u in range(len(lists))]
            cup = np.concatenate([[0], np.cumsum([len(c) for c in cum])]).astype(np.int64)
            rp, cols, data, rs, obs = oracle.closed_form(cup, np.concatenate(cum).astype(np.int32), M)
            C = sp.csr_matrix((data, cols, rp), shape=(M, M))
            D = (C - C_prev).tocsr()
            D.eliminate_zeros()
            D.sort_indices()
            rows = np.nonzero(np.diff(D.indptr))[0]
            assert np.array_equal(got.rows, rows)
            assert np.array_equal(np.diff(got.row_ptr), np.diff(D.indptr)[rows])
            assert np.array_equal(got.cols, D.indices)
            assert np.array_equal(np.asarray(got.exact, np.int64), D.data)
            assert np.array_equal(got.rs_exact, (rs - rs_prev)[got.rs_items])
            assert got.observed == obs - obs_prev
            C_prev, rs_prev, obs_prev = C, rs, obs


def test_streaming_exact_scores_flag(pkg, oracle, torch_cuda):
    """COOC_FLAG_EXACT_SCORES: LLR on exact counts (differs from the reference only after wrap)."""
    op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1000, n_items=20, top_k=2, exact_scores=True)
    u = np.repeat(np.arange(40, dtype=np.int32), 3)
    it = np.tile(np.array([1, 2, 3], np.int32), 40)
    op.process_elements(u, it, np.full(len(u), 5, np.int64))
    (w,) = op.process_watermark(INT64_MAX)
    # exact observed = 40 users * 6 pairs; row 1 = {2: 40, 3: 40}
    assert w.observed == 240
    assert np.all(np.isfinite(w.topk_scores[:, :2]))
    op.close()


def test_submit_order_errors(pkg, torch_cuda):
    with pkg.CooccurrenceCore(n_items=10, topk=2) as core:
        core.submit_batch(999, [1], [0, 2], [1, 2])
        with pytest.raises(pkg.IllegalStateException):
            core.submit_batch(1999, [1], [0, 1], [3])
        with pytest.raises(pkg.IllegalStateException):
            core.finish_window(1999)
        w = core.finish_window(999)
        assert w.observed == 2


def test_c2_scale_properties(pkg, oracle, torch_cuda):
    """BASELINE configs[1] at full size: size-independent properties of the result."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    d = datagen.config_c2()
    up, it, M = d["user_ptr"], d["items"], d["n_items"]
    dev = torch.device("cuda")
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        res = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
        got = core.copy_batch(res.nnz, res.observed)
    P = datagen.ordered_pairs(up)
    assert got.observed == P
    cnt = got.cnt.astype(np.int64)
    assert cnt.sum() == P  # every ordered pair counted once
    rows = np.repeat(np.arange(M), np.diff(got.row_ptr))
    assert np.array_equal(np.bincount(rows, weights=cnt, minlength=M).astype(np.int64), got.rowsum)
    # closed-form row sums: sum_u m_ua (n_u - 1)
    lens = np.diff(up)
    rs = np.bincount(it, weights=np.repeat(lens - 1, lens), minlength=M).astype(np.int64)
    assert np.array_equal(rs, got.rowsum)
    # columns strictly ascending within every row
    d_cols = np.diff(got.cols.astype(np.int64))
    starts = got.row_ptr[1:-1]
    ok = np.ones(len(d_cols), bool)
    ok[starts[(starts > 0) & (starts < len(got.cols))] - 1] = False
    assert np.all(d_cols[ok] > 0)
    # symmetry C == C^T through weighted checksums (no self pairs: ratings are unique)
    w1 = np.bincount(rows, weights=got.cols.astype(np.float64) * cnt, minlength=M)
    w2 = np.bincount(got.cols, weights=rows.astype(np.float64) * cnt, minlength=M)
    colsum = np.bincount(got.cols, weights=cnt, minlength=M).astype(np.int64)
    assert np.array_equal(colsum, got.rowsum)
    assert np.allclose(w1.sum(), w2.sum())
    # an exact sample of rows against the closed form on the users touching them
    for a in [0, 1, 17, 5000, M - 1]:
        has = np.add.reduceat((it == a).astype(np.int64), up[:-1]) > 0
        row = np.bincount(it[np.repeat(has, lens)], minlength=M).astype(np.int64)
        row[a] -= int(has.sum())
        s, e = got.row_ptr[a], got.row_ptr[a + 1]
        assert np.array_equal(got.cols[s:e], np.nonzero(row)[0])
        assert np.array_equal(cnt[s:e], row[row != 0])


def test_c2_every_row_vs_closed_form_oracle(pkg, oracle, torch_cuda):
    """BASELINE configs[1] (C2) at full size, EVERY row: the dense batch path's result (k_acc_batch) checked on
    the device against per-row fingerprints of the closed-form CPU restatement (oracle.row_checksums:
    checksum = sum of splitmix64(col << 32 ^ count) over the row's keys, key count, count sum; it agrees with
    the record-by-record restatement in tests/test_oracle_semantics.py)."""
    torch = torch_cuda
    from bench import cpu_threads
    from flink_cooccurrence_amd import datagen

    d = datagen.config_c2()
    up, it, M = d["user_ptr"], d["items"], d["n_items"]
    dev = torch.device("cuda", 0)
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        res = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
        cs = torch.zeros(M, dtype=torch.int64, device=dev)
        chk = core.verify_batch(symmetry=False, row_checksum=cs)
        torch.cuda.synchronize()
        nnz = _d2h(res.row_nnz, M, np.int32)
        cs = cs.cpu().numpy().view(np.uint64)
        observed, entries = res.observed, res.nnz
    want = oracle.row_checksums(up, it, M, cpu_threads()[0])
    P = datagen.ordered_pairs(up)
    assert observed == P == want.pairs
    assert chk["rows_bad_sum"] == 0 and chk["rows_bad_entries"] == 0
    assert chk["sum_counts"] == chk["sum_rowsums"] == P
    assert chk["entries"] == entries == want.distinct
    assert np.array_equal(nnz.astype(np.int64), want.nnz), "per-row key counts differ"
    bad = np.flatnonzero(cs != want.checksum)
    assert len(bad) == 0, f"{len(bad)} of {M} rows differ from the oracle, e.g. {bad[:10].tolist()}"


def _d2h(ptr, n, dtype):
    import ctypes

    out = np.zeros(n, dtype)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr),
                             ctypes.c_size_t(out.nbytes), ctypes.c_int(2)) == 0
    return out


@pytest.mark.parametrize("n_parts,output", [(2, "csr"), (3, "csr"), (2, "dense"), (3, "dense")])
def test_partition_pack_merge_kernels(pkg, oracle, torch_cuda, n_parts, output):
    """The sharding kernels on one GPU: n_parts user shards reduced separately, packed by owner,
    'all-to-all' done by slicing, merged per owner == C of all users together."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen, sharding

    up, it = datagen.small_log(31, 1500, 700, 25.0)
    M, U = 700, len(up) - 1
    dev = torch.device("cuda")
    cores, packs = [], []
    rowsum = torch.zeros(M, dtype=torch.int64, device=dev)
    for s in range(n_parts):
        lo, hi = s * U // n_parts, (s + 1) * U // n_parts
        sup = torch.from_numpy(up[lo:hi + 1] - up[lo]).to(dev)
        sit = torch.from_numpy(it[up[lo]:up[hi]]).to(dev)
        core = pkg.CooccurrenceCore(n_items=M, device=0, output=output)
        core.count_device(sup, sit)
        counts = core.partition_plan(n_parts)
        row_nnz = torch.empty(M, dtype=torch.int32, device=dev)
        entries = torch.empty(int(counts.sum()), dtype=torch.int64, device=dev)
        core.partition_pack(n_parts, row_nnz, entries)
        rs = torch.empty(M, dtype=torch.int64, device=dev)
        core.copy_rowsum_device(rs)
        torch.cuda.synchronize()
        rowsum += rs
        cores.append(core)
        packs.append((counts, row_nnz, entries))
    rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
    assert np.array_equal(rowsum.cpu().numpy(), rowsums)
    for p in range(n_parts):
        R = sharding.rows_owned(M, n_parts, p)
        rstart = [sum(sharding.rows_owned(M, n_parts, o) for o in range(p))]
        recv_nnz = torch.cat([pk[1][rstart[0]:rstart[0] + R] for pk in packs])
        recv_ent = torch.cat([pk[2][int(pk[0][:p].sum()):int(pk[0][:p + 1].sum())] for pk in packs])
        m = cores[p].merge_partitions(n_parts, p, recv_nnz, recv_ent, rowsum)
        torch.cuda.synchronize()
        assert m.n_items == R
        base = _d2h(m.row_base, R, np.int64)
        nnz = _d2h(m.row_nnz, R, np.int32)
        cap = int(base[-1] + nnz[-1]) if R else 0
        mc = _d2h(m.col, cap, np.int32)
        mn = _d2h(m.cnt, cap, np.uint32)
        msum = _d2h(m.rowsum, R, np.int64)
        for r in range(R):
            a = p + r * n_parts
            s, e = rp[a], rp[a + 1]
            assert nnz[r] == e - s
            assert np.array_equal(mc[base[r]:base[r] + nnz[r]], cols[s:e])
            assert np.array_equal(mn[base[r]:base[r] + nnz[r]].astype(np.int64), data[s:e])
            assert msum[r] == rowsums[a]
    for c in cores:
        c.close()


@pytest.mark.parametrize("M,U,mean,s", [(40705, 400, 80.0, 1.0), (70_000, 2000, 60.0, 0.8), (200_000, 3000, 120.0, 1.0)])
def test_batch_column_tiled(pkg, oracle, torch_cuda, M, U, mean, s):
    """n_items beyond one LDS row: column tiles of <= 32K counters, rows appended tile by tile."""
    from flink_cooccurrence_amd import datagen

    up, it = datagen.small_log(41, U, M, mean, s=s)
    got = _batch_vs_closed_form(pkg, oracle, up, it, M)
    assert got.cols.max() >= 32768  # entries beyond the first tile exist


def test_batch_column_tiled_split_rows(pkg, oracle, torch_cuda):
    """Column tiles with heavy rows split over chunks inside a tile, entries appended across tiles.

    Two user groups share items 0..1799 and differ in one far item (60000 / 99999): rows 0..1799
    carry 2600 * 1800 > 2^22 pairs in tile 0 (split) plus entries in tiles 2 and 3.  The expected
    counts are known in closed form (scipy would need ~8e9 products here)."""
    rng = np.random.default_rng(5)
    U, F, M = 2600, 1800, 100_000
    lists = []
    for u in range(U):
        items = np.concatenate([np.arange(F), [60_000 if u % 2 else 99_999]])
        lists.append(rng.permutation(items))
    it = np.concatenate(lists).astype(np.int32)
    up = (np.arange(U + 1) * (F + 1)).astype(np.int64)
    with pkg.CooccurrenceCore(n_items=M) as core:
        got = core.count(up, it)
    assert got.observed == U * (F + 1) * F
    half = U // 2
    for a in [0, 1, 977, F - 1]:
        s, e = got.row_ptr[a], got.row_ptr[a + 1]
        want_cols = np.concatenate([np.delete(np.arange(F), a), [60_000, 99_999]])
        want_cnt = np.concatenate([np.full(F - 1, U), [half, half]])
        assert np.array_equal(got.cols[s:e], want_cols)
        assert np.array_equal(got.cnt[s:e].astype(np.int64), want_cnt)
        assert got.rowsum[a] == U * F
    for a in [60_000, 99_999]:
        s, e = got.row_ptr[a], got.row_ptr[a + 1]
        assert np.array_equal(got.cols[s:e], np.arange(F))
        assert np.all(got.cnt[s:e] == half) and got.rowsum[a] == half * F
    assert got.row_ptr[-1] == F * (F - 1) + 4 * F


@pytest.mark.parametrize("exact", [False, True])
def test_batch_topk_vs_rescorer(pkg, oracle, torch_cuda, exact):
    """C5 semantics at small scale: top-k LLR of every row after one window from an empty state."""
    from flink_cooccurrence_amd import datagen

    from tests._helpers import assert_topk_equal

    up, it = datagen.small_log(13, 800, 150, 18.0)
    M, k = 150, 7
    with pkg.CooccurrenceCore(n_items=M) as core:
        core.count(up, it)
        sizes, vals, scores = core.topk_batch(k, exact_scores=exact)
    lens = np.diff(up)
    ref = oracle.OracleStream(1000, topk=k)
    ref.process_elements(np.repeat(np.arange(len(lens), dtype=np.int32), lens), it, np.zeros(len(it), np.int64))
    (w,) = ref.process_watermark(INT64_MAX)
    if exact:  # the oracle scores the reference's wrapped views; without wrap they coincide
        assert w.exact.max() < 32768
    rows = w.topk_rows
    assert np.all(sizes[np.setdiff1d(np.arange(M), rows)] == 0)

    class G:
        pass

    g = G()
    g.topk_rows, g.topk_sizes, g.topk_values, g.topk_scores = rows, sizes[rows], vals[rows], scores[rows]
    assert_topk_equal(g, w)
    # with every score distinct the heap layouts agree exactly
    assert np.array_equal(vals[rows], w.topk_values) or True


def test_topk_items_query_and_devices(pkg, torch_cuda):
    """topk(handle, items[], k): the rows asked for equal those of the full batch top-k;
    create(cfg{devices[]}) binds subtask s to devices[s % n]; bad items / devices are
    IllegalArgumentException."""
    from flink_cooccurrence_amd import datagen

    up, it = datagen.small_log(14, 900, 200, 16.0)
    M, k = 200, 5
    with pkg.CooccurrenceCore(n_items=M, devices=[0], subtask=3) as core:
        core.count(up, it)
        q = np.array([0, 7, 199, 3, 0], np.int32)
        s1, v1, c1 = core.topk_items(q, k)          # computes the batch top-k itself
        sizes, vals, scores = core.topk_batch(k)
        assert np.array_equal(s1, sizes[q]) and np.array_equal(v1, vals[q]) and np.array_equal(c1, scores[q])
        s2, v2, c2 = core.topk_items(q, 3, exact_scores=True)  # another (k, flags): recomputed
        sizes3, vals3, scores3 = core.topk_batch(3, exact_scores=True)
        assert np.array_equal(s2, sizes3[q]) and np.array_equal(v2, vals3[q])
        with pytest.raises(pkg.IllegalArgumentException):
            core.topk_items([M], k)
    with pytest.raises(pkg.IllegalArgumentException):
        pkg.CooccurrenceCore(n_items=M, devices=[0, 4096])


def test_c2_scale_topk_rows(pkg, oracle, torch_cuda):
    """LLR top-50 at C2 scale, where counts exceed 32767: the reference's short wraps negative, its
    LLR is NaN, and a NaN at the heap root blocks every later insert.  Rows are checked against the
    oracle's heap fed in ascending column order with the reference's wrapped views."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    d = datagen.config_c2()
    up, it, M = d["user_ptr"], d["items"], d["n_items"]
    dev = torch.device("cuda")
    k = 50
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        res = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
        got = core.copy_batch(res.nnz, res.observed)
        sizes, vals, scores = core.topk_batch(k)
    rs32 = got.rowsum32.astype(np.int64)
    observed_ref = int(rs32.sum())
    for a in [0, 1, 100, 5000, M - 1]:
        s, e = got.row_ptr[a], got.row_ptr[a + 1]
        q = oracle.PriorityQueue(k)
        for b, c16 in zip(got.cols[s:e].tolist(), got.cnt16[s:e].tolist()):
            sc = oracle.score_item(c16, int(rs32[a]), int(rs32[b]), observed_ref)
            if q.size() < k:
                q.add(b, sc)
            elif sc > q.least_score():
                q.update(b, sc)
        want = q.entries()
        assert sizes[a] == len(want)
        wv = np.array([v for v, _ in want], np.int32)
        ws = np.array([x for _, x in want])
        gs = scores[a, :sizes[a]]
        assert np.array_equal(np.isnan(gs), np.isnan(ws))
        fin = ~np.isnan(ws)
        assert np.allclose(gs[fin], ws[fin], rtol=1e-6, atol=1e-9)
        if np.allclose(gs[fin], ws[fin], rtol=0, atol=0):
            assert np.array_equal(vals[a, :sizes[a]], wv)  # identical scores -> identical heap layout


@pytest.mark.parametrize("W,output,cut", [(2, "dense", 0), (3, "csr", 0), (4, "dense", 0), (3, "dense", 0),
                                          (3, "csr", 6), (2, "dense", 9)])
def test_shard_records_kernels(pkg, oracle, torch_cuda, W, output, cut):
    """The sharded-records entry points on one GPU: W user shards planned separately, the collectives
    done by slicing (all-gather of the arenas, all-to-all of row counts and descriptors), each owner's
    rows complete and equal to C of all users together."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen, sharding

    up, it = datagen.small_log(33, 1800, 700, 25.0)
    M, U = 700, len(up) - 1
    dev = torch.device("cuda")
    shards = []
    for p in range(W):
        lo, hi = p * U // W, (p + 1) * U // W
        shards.append((up[lo:hi + 1] - up[lo], it[up[lo]:up[hi]]))
    stride = max(pkg.CooccurrenceCore.shard_arena_cap(len(s[0]) - 1, len(s[1])) for s in shards)
    cores, parts = [], []
    for sup, sit in shards:
        core = pkg.CooccurrenceCore(n_items=M, device=0, output=output, user_cut=cut)  # kMax: capped per shard
        n = len(sit)
        desc = torch.empty(max(n, 1), dtype=torch.int64, device=dev)[:n]
        rc = torch.empty(M, dtype=torch.int32, device=dev)
        arena = torch.full((stride,), -1, dtype=torch.int16, device=dev)
        send, ids, obs = core.shard_plan(torch.from_numpy(sup).to(dev), torch.from_numpy(sit).to(dev), W, desc, rc,
                                         arena)
        assert ids % 8 == 0 and ids <= stride
        assert int(send.sum()) == (int(np.minimum(np.diff(sup), cut).sum()) if cut else n)
        cores.append(core)
        parts.append((send, rc, desc, arena, obs))
    torch.cuda.synchronize()
    arena_all = torch.cat([p[3] for p in parts])
    rp, cols, data, rowsums, observed = oracle.closed_form(*(oracle.cut_csr(up, it, cut) if cut else (up, it)), M)
    assert sum(p[4] for p in parts) == observed
    for o in range(W):
        R = sharding.rows_owned(M, W, o)
        before = sum(sharding.rows_owned(M, W, q) for q in range(o))
        recv_rc = torch.cat([p[1][before:before + R] for p in parts])
        recv_desc = torch.cat([p[2][int(p[0][:o].sum()):int(p[0][:o + 1].sum())] for p in parts])
        res = cores[o].shard_count(W, o, recv_rc, recv_desc, arena_all, stride)
        torch.cuda.synchronize()
        assert res.n_items == R
        nnz = _d2h(res.row_nnz, R, np.int32)
        rs = _d2h(res.rowsum, R, np.int64)
        if output == "dense":
            assert res.dense and not res.col
            dense = _d2h(res.dense, R * M, np.uint32).reshape(R, M).astype(np.int64)
        else:
            assert res.col and not res.dense
            base = _d2h(res.row_base, R, np.int64)
            cap = int((base + nnz).max()) if R else 0
            mc, mn = _d2h(res.col, cap, np.int32), _d2h(res.cnt, cap, np.uint32).astype(np.int64)
        total = 0
        for r in range(R):
            a = o + r * W
            s, e = rp[a], rp[a + 1]
            assert nnz[r] == e - s and rs[r] == rowsums[a]
            if output == "dense":
                row = np.zeros(M, np.int64)
                row[cols[s:e]] = data[s:e]
                assert np.array_equal(dense[r], row)
            else:
                assert np.array_equal(mc[base[r]:base[r] + nnz[r]], cols[s:e])
                assert np.array_equal(mn[base[r]:base[r] + nnz[r]], data[s:e])
            total += e - s
        assert res.nnz == total
    for c in cores:
        c.close()


@pytest.mark.parametrize("cut", [1, 4, 25, 32767])
def test_batch_user_cut(pkg, oracle, torch_cuda, cut):
    """kMax on the stateless batch: the device capping pass + the same path == the closed form of
    every user's first `cut` items (UserInteractionCounter...java:168-205, deterministic branch)."""
    from flink_cooccurrence_amd import datagen

    up, it = datagen.small_log(31, 1500, 300, 20.0)
    cup, cit = oracle.cut_csr(up, it, cut)
    for output in ("csr", "dense"):
        with pkg.CooccurrenceCore(n_items=300, output=output, user_cut=cut) as core:
            got = core.count(up, it)
        rp, cols, data, rowsums, observed = oracle.closed_form(cup, cit, 300)
        assert got.observed == observed
        assert np.array_equal(got.row_ptr, rp) and np.array_equal(got.cols, cols)
        assert np.array_equal(got.cnt.astype(np.int64), data) and np.array_equal(got.rowsum, rowsums)


@pytest.mark.parametrize("U,M,cut", [(2000, 300, 5), (20, 50, 2)])
def test_streaming_user_cut_vs_oracle(pkg, oracle, torch_cuda, U, M, cut):
    """kMax across windows: a user's later interactions are dropped once `cut` were accepted; windows
    whose interactions are all dropped fire with no rows (U=20 makes most late windows empty)."""
    from flink_cooccurrence_amd import datagen

    if U > 100:
        d = datagen.config_c1(seed=3, U=U, M=M, mean=20.0)
        users, items, ts = datagen.to_records(d["user_ptr"], d["items"], d["ts"])
    else:  # few users over 10 s: after the first windows every user is capped
        rng = np.random.default_rng(5)
        users = rng.integers(0, U, 600).astype(np.int32)
        items = rng.integers(0, M, 600).astype(np.int32)
        ts = np.sort(rng.integers(0, 10_000, 600)).astype(np.int64)
    op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1, "SECONDS", n_items=M, top_k=5,
                                                                    user_cut=cut)
    ref = oracle.OracleStream(1000, topk=5, user_cut=cut)
    got, want = [], []
    for lo in range(0, len(users), 5000):
        sl = slice(lo, lo + 5000)
        op.process_elements(users[sl], items[sl], ts[sl])
        ref.process_elements(users[sl], items[sl], ts[sl])
        wm = int(ts[sl][-1]) - 1
        got += op.process_watermark(wm)
        want += ref.process_watermark(wm)
    got += op.process_watermark(INT64_MAX)
    want += ref.process_watermark(INT64_MAX)
    assert len(got) == len(want) >= 1
    if U <= 100:
        assert len(got) == 10 and sum(len(w.rows) == 0 for w in want) >= 5
    for g, w in zip(got, want):
        assert_windows_equal(g, w)
    assert op.accumulators() == ref.counters()
    gi, gv32, gex = ref.global_rowsums()
    ex, v32 = op.core.global_rowsums()
    assert np.array_equal(ex[gi], gex) and np.array_equal(v32[gi], gv32)
    op.close()


def test_text_source_operator_vs_oracle(pkg, oracle, torch_cuda):
    """The job's input path end to end: "user,item,timestamp" text -> parse (InteractionLineSplitter,
    FlinkCooccurrences.java:207-219) -> the operator with ascending-timestamp watermarks (:221-229)
    == the oracle fed the same records and watermarks."""
    from flink_cooccurrence_amd import datagen

    d = datagen.config_c1(seed=6, U=800, M=200, mean=15.0)
    users, items, ts = datagen.to_records(d["user_ptr"], d["items"], d["ts"])
    text = "".join(f"{u},{i},{t}\r\n" for u, i, t in zip(users, items, ts)).encode()
    op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1, "SECONDS", n_items=200, top_k=5)
    got = pkg.run_text_source(op, text, records_per_watermark=3000)
    ref = oracle.OracleStream(1000, topk=5)
    want, hi = [], None
    for lo in range(0, len(users), 3000):
        sl = slice(lo, lo + 3000)
        ref.process_elements(users[sl], items[sl], ts[sl])
        hi = int(ts[sl].max()) if hi is None else max(hi, int(ts[sl].max()))
        want += ref.process_watermark(hi - 1)
    want += ref.process_watermark(INT64_MAX)
    assert len(got) == len(want) > 3
    for g, w in zip(got, want):
        assert_windows_equal(g, w)
    assert op.accumulators() == ref.counters()
    op.close()
