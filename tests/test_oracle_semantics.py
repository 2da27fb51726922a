"""The oracle against the hand-derived micro-logs and its independent restatements (CPU)."""
import numpy as np
import pytest
import scipy.sparse as sp

from tests._helpers import (INT64_MAX, as_int_keys, micro_csr, micro_events, micro_logs, run_events, window_rows,
                            window_rows16)


@pytest.mark.parametrize("log", micro_logs(), ids=lambda l: l["name"])
def test_micro_logs(oracle, log):
    if log.get("closed_form_only"):
        up, it = micro_csr(log)
        M = int(it.max()) + 1
        rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
        w = log["windows"][0]
        C = sp.csr_matrix((data, cols, rp), shape=(M, M))
        for a, row in as_int_keys(w["rows"]).items():
            for b, v in row.items():
                assert C[a, b] == v
                assert oracle.to_i16(v) == as_int_keys(w["rows16"])[a][b]
        for a, v in as_int_keys(w["rowsums"]).items():
            assert rowsums[a] == v
            assert oracle.to_i32(v) == as_int_keys(w["rowsums32"])[a]
        assert observed == w["observed"]
        return
    s = oracle.OracleStream(log["window_ms"], topk=3)
    fired = run_events(micro_events(log), s.process_elements, s.process_watermark)
    assert len(fired) == len(log["windows"])
    for got, want in zip(fired, log["windows"]):
        assert got.ts == want["ts"]
        assert window_rows(got) == as_int_keys(want["rows"])
        if "rows16" in want:
            assert window_rows16(got) == as_int_keys(want["rows16"])
        assert dict(zip(got.rs_items.tolist(), got.rs_exact.tolist())) == as_int_keys(want["rowsums"])
        assert got.observed == want["observed"]
    c = s.counters()
    assert c["UserInteractionCounterLateElements"] == log["late"]
    if "global_rows" in log:
        rows, rp, cols, exact, _ = s.global_rows()
        g = {int(a): dict(zip(cols[rp[r]:rp[r + 1]].tolist(), exact[rp[r]:rp[r + 1]].tolist()))
             for r, a in enumerate(rows)}
        assert g == as_int_keys(log["global_rows"])
        items, v32, ex = s.global_rowsums()
        assert dict(zip(items.tolist(), ex.tolist())) == as_int_keys(log["global_rowsums"])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_three_restatements_agree(oracle, seed):
    rng = np.random.default_rng(seed)
    U, M = 60, 15
    lens = rng.integers(1, 10, U)
    up = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    it = rng.integers(0, M, up[-1]).astype(np.int32)
    dense, rs, obs = oracle.batch_dense(up, it, M)
    rp, cols, data, rs2, obs2 = oracle.closed_form(up, it, M)
    assert np.array_equal(sp.csr_matrix((data, cols, rp), shape=(M, M)).toarray(), dense)
    assert np.array_equal(rs, rs2) and obs == obs2
    counts, rsd, obs3 = oracle.literal_python([it[up[u]:up[u + 1]].tolist() for u in range(U)])
    D = np.zeros((M, M), np.int64)
    for (a, b), v in counts.items():
        D[a, b] = v
    assert np.array_equal(D, dense) and obs3 == obs


def test_streaming_windows_sum_to_closed_form(oracle):
    """Per-window deltas summed over windows == C of the whole log; global rows == that sum."""
    rng = np.random.default_rng(11)
    U, M, n = 40, 25, 900
    users = rng.integers(0, U, n).astype(np.int32)
    items = rng.integers(0, M, n).astype(np.int32)
    ts = np.sort(rng.integers(0, 10_000, n)).astype(np.int64)
    s = oracle.OracleStream(1000, topk=5)
    s.process_elements(users, items, ts)
    wins = s.process_watermark(INT64_MAX)
    assert [w.ts for w in wins] == sorted({int(oracle.window_max_ts(t, 1000)) for t in ts})
    tot = np.zeros((M, M), np.int64)
    for w in wins:
        for r, a in enumerate(w.rows):
            tot[a, w.cols[w.row_ptr[r]:w.row_ptr[r + 1]]] += w.exact[w.row_ptr[r]:w.row_ptr[r + 1]]
    order = np.lexsort((np.arange(n), users))  # per-user arrival order
    lens = np.bincount(users, minlength=U)
    up = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    rp, cols, data, rs, obs = oracle.closed_form(up, items[order], M)
    assert np.array_equal(tot, sp.csr_matrix((data, cols, rp), shape=(M, M)).toarray())
    rows, grp, gcols, gex, g16 = s.global_rows()
    G = np.zeros((M, M), np.int64)
    for r, a in enumerate(rows):
        G[a, gcols[grp[r]:grp[r + 1]]] = gex[grp[r]:grp[r + 1]]
    assert np.array_equal(G, tot)
    c = s.counters()
    assert c["UserInteractionCounterObservedCooccurrences"] == obs == c["rescorer_observed"]
    assert c["ItemRowRescorerRescoredItems"] == sum(len(w.rows) for w in wins)


def test_window_assignment_matches_flink(oracle):
    # TumblingEventTimeWindows offset 0: [k*size, (k+1)*size), maxTimestamp = end - 1
    assert oracle.window_max_ts(0, 1000) == 999
    assert oracle.window_max_ts(999, 1000) == 999
    assert oracle.window_max_ts(1000, 1000) == 1999
    assert oracle.window_max_ts(-1, 1000) == -1


@pytest.mark.parametrize("cut", [1, 3, 7])
def test_user_cut_restatements_agree(oracle, cut):
    """kMax (UserInteractionCounter...java:168-205, deterministic branch): the record-by-record
    oracle over several windows == the literal expansion of every user's first `cut` interactions ==
    the closed form of the capped CSR."""
    rng = np.random.default_rng(20 + cut)
    U, M, n = 30, 12, 700
    users = rng.integers(0, U, n).astype(np.int32)
    items = rng.integers(0, M, n).astype(np.int32)
    ts = np.sort(rng.integers(0, 8_000, n)).astype(np.int64)
    s = oracle.OracleStream(1000, topk=3, user_cut=cut)
    s.process_elements(users, items, ts)
    wins = s.process_watermark(INT64_MAX)
    tot = np.zeros((M, M), np.int64)
    for w in wins:
        for r, a in enumerate(w.rows):
            tot[a, w.cols[w.row_ptr[r]:w.row_ptr[r + 1]]] += w.exact[w.row_ptr[r]:w.row_ptr[r + 1]]
    order = np.lexsort((np.arange(n), users))
    lens = np.bincount(users, minlength=U)
    up = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    it = items[order]
    counts, _, obs_lit = oracle.literal_python([it[up[u]:up[u + 1]].tolist() for u in range(U)], user_cut=cut)
    D = np.zeros((M, M), np.int64)
    for (a, b), v in counts.items():
        D[a, b] = v
    cup, cit = oracle.cut_csr(up, it, cut)
    assert np.diff(cup).max() <= cut
    rp, cols, data, rs, obs = oracle.closed_form(cup, cit, M)
    assert np.array_equal(tot, D)
    assert np.array_equal(D, sp.csr_matrix((data, cols, rp), shape=(M, M)).toarray())
    assert s.counters()["UserInteractionCounterObservedCooccurrences"] == obs == obs_lit
    with pytest.raises(ValueError):
        oracle.OracleStream(1000, user_cut=40000)  # a Java short


@pytest.mark.parametrize("seed,U,M", [(4, 300, 40), (5, 2000, 5000), (6, 1, 3), (7, 0, 5)])
def test_row_checksum_oracles_agree(oracle, seed, U, M):
    """The per-row fingerprints (checksum, keys, count sum) of the record-by-record restatement
    (count_batch_mt_rows), of the fast closed-form restatement (row_checksums: the benchmark's
    exactness check at full size) and of scipy's A^T A - diag(colsum A) agree; repeats included."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 30, U)
    up = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    it = (rng.zipf(1.3, int(up[-1])) % M).astype(np.int32)
    rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
    want = oracle.csr_row_checks(rp, cols, data)
    for threads in (1, 3):
        for got in (oracle.count_batch_mt_rows(up, it, M, threads), oracle.row_checksums(up, it, M, threads)):
            assert np.array_equal(got.checksum, want.checksum)
            assert np.array_equal(got.nnz, want.nnz)
            assert np.array_equal(got.rowsum, rowsums) and np.array_equal(want.rowsum, rowsums)
            assert got.distinct == len(cols) and got.pairs == observed


def test_row_checksum_detects_a_changed_count(oracle):
    up = np.array([0, 3, 5], np.int64)
    it = np.array([1, 2, 2, 1, 0], np.int32)
    rp, cols, data, _, _ = oracle.closed_form(up, it, 3)
    base = oracle.csr_row_checks(rp, cols, data).checksum
    data2 = data.copy()
    data2[0] += 1
    assert not np.array_equal(oracle.csr_row_checks(rp, cols, data2).checksum, base)
    cols2 = cols.copy()
    cols2[-1] = 0 if cols2[-1] else 1
    assert not np.array_equal(oracle.csr_row_checks(rp, cols2, data).checksum, base)
