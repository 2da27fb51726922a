"""The large-universe path (n_items >= 40,320: cooc_sparse.hip) against the closed form and against
rows summed directly from the users' lists.  Needs an MI355X.

Covers every chunk kind of k_sp_main: hash chunks, dense tiles, gather mode (rows of many chunks whose
tails go through the per-workgroup buckets), split rows (shares of a row's contributions into a staging
row, finalize with the uint32 overflow check), and the C3 log itself at 1/64 of the 1B-interaction
config through size-independent properties (observed == P, sum of row sums == P, symmetry of sampled
entries, sorted keys) plus exact sampled rows.  Bar: bit-exact.
"""
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


def _d2h(ptr, n, dtype, offset=0):
    out = np.zeros(n, dtype)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        src = ctypes.c_void_p(ptr + offset * out.itemsize)
        assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), src, ctypes.c_size_t(out.nbytes), ctypes.c_int(2)) == 0
    return out


class _Rows:
    """Rows of a count_device result, read back one at a time."""

    def __init__(self, res, M):
        self.res, self.M = res, M
        self.base = _d2h(res.row_base, M, np.int64)
        self.nnz = _d2h(res.row_nnz, M, np.int32)
        self.rowsum = _d2h(res.rowsum, M, np.int64)

    def row(self, a):
        """Row a in ascending id order (the device row's own order -- hot items first after the
        large-universe renumbering, cooc.h COOC_FLAG_COLUMN_ORDER -- is checked by cooc_verify_batch)."""
        n, b = int(self.nnz[a]), int(self.base[a])
        c, v = _d2h(self.res.col, n, np.int32, b), _d2h(self.res.cnt, n, np.uint32, b).astype(np.int64)
        o = np.argsort(c, kind="stable")
        return c[o], v[o]


class _Brute:
    """C[a, :] = sum over the users u holding a of m_u(a) * (u's list as counts), minus m_u(a) at a
    (NonSampled...java:129-161 summed per row; the closed form of SURVEY.md §0.3 restricted to a)."""

    def __init__(self, up, it, M):
        self.up, self.it, self.M = np.asarray(up, np.int64), np.asarray(it, np.int64), M
        self.lens = np.diff(self.up)
        self.users = np.repeat(np.arange(len(self.lens)), self.lens)
        self.order = np.argsort(self.it, kind="stable")
        self.sorted = self.it[self.order]

    def row(self, a):
        lo, hi = np.searchsorted(self.sorted, [a, a + 1])
        us, mult = np.unique(self.users[self.order[lo:hi]], return_counts=True)
        if len(us) == 0:
            return np.zeros(0, np.int32), np.zeros(0, np.int64)
        starts, lens = self.up[us], self.lens[us]
        idx = np.repeat(starts - np.cumsum(np.concatenate([[0], lens[:-1]])), lens) + np.arange(lens.sum())
        row = np.bincount(self.it[idx], weights=np.repeat(mult, lens).astype(np.float64), minlength=self.M)
        row = np.rint(row).astype(np.int64)
        row[a] -= int(mult.sum())
        nz = np.nonzero(row)[0]
        return nz.astype(np.int32), row[nz]


def _structured_log(U=20_000, F=200, K=100, R=300, M=300_000, seed=11):
    """Users hold the shared items 0..F-1 (rows of U * ~(F + R) > 2^23 pairs: split rows), every third
    user also K medium items F..F+K-1 (rows of ~4e6 pairs, tile 0 dense plus ~8 dense tail tiles:
    gather mode), and R random tail items (with replacement) in [32768, M)."""
    rng = np.random.default_rng(seed)
    lists = []
    for u in range(U):
        parts = [np.arange(F), rng.integers(32768, M, R)]
        if u % 3 == 0:
            parts.append(np.arange(F, F + K))
        lists.append(rng.permutation(np.concatenate(parts)))
    up = np.concatenate([[0], np.cumsum([len(x) for x in lists])]).astype(np.int64)
    return up, np.concatenate(lists).astype(np.int32), M


def _check_rows(rows, brute, sample):
    for a in sample:
        gc, gn = rows.row(int(a))
        wc, wn = brute.row(int(a))
        assert np.array_equal(gc, wc), f"row {a}: key set differs"
        assert np.array_equal(gn, wn), f"row {a}: counts differ"
        assert int(gn.sum()) == int(rows.rowsum[a])


@pytest.mark.parametrize("planner", ["auto", "sort"])
def test_gather_and_split_rows_vs_brute(pkg, torch_cuda, planner):
    """planner="sort": the split rows as usual, every whole row through the sort + segmented-reduce path."""
    torch = torch_cuda
    up, it, M = _structured_log()
    dev = torch.device("cuda")
    with pkg.CooccurrenceCore(n_items=M, device=0, planner=planner) as core:
        res = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
        torch.cuda.current_stream().synchronize()
        lens = np.diff(up)
        assert res.observed == int(np.sum(lens * (lens - 1)))
        rows = _Rows(res, M)
        assert int(rows.nnz.sum()) == res.nnz
        assert int(rows.rowsum.sum()) == res.observed
        brute = _Brute(up, it, M)
        rng = np.random.default_rng(3)
        tail = np.unique(it[it >= 32768])
        sample = np.concatenate([[0, 1, 57, 199], [200, 201, 250, 299], rng.choice(tail, 40, replace=False),
                                 [300, 32767]])
        _check_rows(rows, brute, sample)
        if planner == "sort":
            assert core.last_sort_rows()[0] == int(np.count_nonzero(rows.nnz)) - 200  # all but the 200 split rows


def test_small_row_full_radix_blocks_vs_closed_form(pkg, oracle, torch_cuda):
    """k_sp_small's LSD radix sort (rows of 257..4,096 pairs, 512-thread workgroups: a wave ranks 512 positions)
    when whole 512-position blocks share one digit: row a = 0x3F80 (digit 0 in pass 0, digit 127 = bits 7..13
    in pass 1) holds 2,200 copies of its own column (600 users [a, x], 400 users [a, a, x]), so in pass 1 the
    last key of a full wave block has digit 127 at rank 511 -- the value the sort once used as its "no key"
    marker, which left a stale LDS word in the sorted row.  The whole CSR against the closed form."""
    rng = np.random.default_rng(5)
    M, a = 100_000, 0x3F80
    xs = rng.choice(np.arange(20_000, M), 1000, replace=False)
    xs = xs[(xs & 127) != 0][:1000]
    lists = [[a, int(x)] for x in xs[:600]] + [[a, a, int(x)] for x in xs[600:]]
    up = np.concatenate([[0], np.cumsum([len(x) for x in lists])]).astype(np.int64)
    it = np.concatenate([np.array(x, np.int32) for x in lists])
    lens = np.diff(up)
    W_a = int(np.sum(lens[[a in x for x in lists]] * np.array([x.count(a) for x in lists])))
    assert 256 < W_a <= 4096  # k_sp_small's row size
    with pkg.CooccurrenceCore(n_items=M) as core:
        got = core.count(up, it)
    rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
    assert got.observed == observed
    assert np.array_equal(got.row_ptr, rp)
    assert np.array_equal(got.cols, cols)
    assert np.array_equal(got.cnt.astype(np.int64), data)
    assert np.array_equal(got.rowsum, rowsums)


@pytest.mark.parametrize("permute", [False, True])
@pytest.mark.parametrize("planner", ["auto", "sort"])
def test_c3_shape_vs_closed_form(pkg, oracle, torch_cuda, planner, permute):
    """The first 1,500 users of the shard-invariant C3 log (1e6 items): the whole CSR vs scipy, through the
    LDS hash / dense-tile chunks and through the sort + segmented-reduce path (k_srb_row, k_sp_small,
    k_sp_tiny); with item ids permuted, through the column relabel as well."""
    from flink_cooccurrence_amd import datagen

    up, it = datagen.c3_users(0, 1500, permute=permute)
    M = datagen.C3_ITEMS
    with pkg.CooccurrenceCore(n_items=M, planner=planner) as core:
        got = core.count(up, it)
        if planner == "sort":
            assert core.last_sort_rows()[0] == len(np.unique(it))
    rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
    assert got.observed == observed
    assert np.array_equal(got.row_ptr, rp)
    assert np.array_equal(got.cols, cols)
    assert np.array_equal(got.cnt.astype(np.int64), data)
    assert np.array_equal(got.rowsum, rowsums)


@pytest.mark.parametrize("permute", [False, True])
def test_any_order_rows_vs_closed_form(pkg, oracle, torch_cuda, permute):
    """COOC_FLAG_ANY_ORDER (hash chunks emitted in slot order, no column ranking) on 3,000 users of the C3 log:
    every device row holds the closed form's keys and counts (as a set), the host copy comes out sorted and
    equal to the closed form, the in-range row copies too, cooc_verify_batch passes without an order check,
    the top-k heaps score the same entries (the sorted score lists equal the ordered run's), and the
    partial-row partition refuses the result."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    up, it = datagen.c3_users(0, 3000, permute=permute)
    M = datagen.C3_ITEMS
    rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
    dev = torch.device("cuda")
    k = 10
    tops = []
    for any_order in (False, True):
        with pkg.CooccurrenceCore(n_items=M, device=0, any_order=any_order) as core:
            res = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
            torch.cuda.current_stream().synchronize()
            chk = core.verify_batch()
            assert chk["rows_bad_sum"] == 0 and chk["rows_bad_entries"] == 0
            assert chk["sum_counts"] == chk["sum_rowsums"] == observed
            rows = _Rows(res, M)
            for a in np.flatnonzero(np.diff(rp))[::37]:
                c, n = rows.row(int(a))  # (sorted here: the device order is free)
                assert np.array_equal(c, cols[rp[a]:rp[a + 1]]) and np.array_equal(n, data[rp[a]:rp[a + 1]])
            got = core.copy_batch(res.nnz, res.observed)
            assert np.array_equal(got.row_ptr, rp) and np.array_equal(got.cols, cols)
            assert np.array_equal(got.cnt.astype(np.int64), data) and np.array_equal(got.rowsum, rowsums)
            r0, r1 = 0, 50_000
            e0, e1 = rp[r0], rp[r1]
            cc, vv, _ = core.copy_batch_range(r0, r1, e1 - e0)
            assert np.array_equal(cc, cols[e0:e1]) and np.array_equal(vv.astype(np.int64), data[e0:e1])
            sample = np.flatnonzero(np.diff(rp))[:200].astype(np.int32)
            sizes, vals, scores = core.topk_items(sample, k)
            tops.append((sizes, [np.sort(scores[i, :s]) for i, s in enumerate(sizes)]))
            if any_order:
                with pytest.raises(pkg.CoocError):
                    core.partition_plan(2)
    assert np.array_equal(tops[0][0], tops[1][0])
    # the same top scores whatever order fed the heaps -- in rows without a NaN score (an int16-wrapped count:
    # NaN compares false in the heap, so which entries stay depends on the feeding order, as in the reference)
    compared = 0
    for x, y in zip(tops[0][1], tops[1][1]):
        if not (np.isnan(x).any() or np.isnan(y).any()):
            assert np.array_equal(x, y)
            compared += 1
    assert compared > 100


def test_c3_sixty_fourth_properties(pkg, torch_cuda):
    """1/64 of C3 (156,250 users, ~1.6e7 interactions, ~4e9 ordered pairs) generated on the GPU:
    observed == P and sum(rowsum) == P from the generator's lengths, sum(row_nnz) == nnz, sampled rows
    sorted and exact (hot, mid and tail items), sampled entries symmetric (C[a, b] == C[b, a])."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    U = datagen.C3_USERS // 64
    M = datagen.C3_ITEMS
    dev = torch.device("cuda")
    up_d, it_d = datagen.c3_users(0, U, device=dev)
    P = datagen.c3_ordered_pairs(0, U)
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        res = core.count_device(up_d, it_d)
        torch.cuda.current_stream().synchronize()
        assert res.observed == P
        rows = _Rows(res, M)
        assert int(rows.rowsum.sum()) == P
        assert int(rows.nnz.sum()) == res.nnz
        up, it = up_d.cpu().numpy(), it_d.cpu().numpy()
        brute = _Brute(up, it, M)
        rng = np.random.default_rng(5)
        sample = np.concatenate([[0, 3, 40, 700], rng.integers(1000, 40_000, 8), rng.integers(40_000, M, 24)])
        _check_rows(rows, brute, sample)
        # symmetry of sampled entries of sampled rows
        for a in rng.integers(0, 50_000, 12):
            ca, na = rows.row(int(a))
            assert np.all(np.diff(ca) > 0)
            for j in rng.integers(0, len(ca), min(8, len(ca))):
                b = int(ca[j])
                cb, nb = rows.row(b)
                k = np.searchsorted(cb, a)
                assert k < len(cb) and cb[k] == a and nb[k] == na[j], f"C[{a},{b}] != C[{b},{a}]"


def test_owned_parts_union_is_whole(pkg, torch_cuda):
    """count_device_owned over 3 parts of a large-universe log on one GPU: every row is counted by
    exactly its owner and equals the unpartitioned result (the multi-GPU row ownership)."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen, sharding

    up, it = datagen.c3_users(0, 3000)
    M = datagen.C3_ITEMS
    dev = torch.device("cuda")
    up_d, it_d = torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev)
    freq = np.bincount(it, minlength=M).astype(np.int64)
    freq_d = torch.from_numpy(freq).to(dev)
    owner_d = sharding.snake_owner(freq_d, 3)
    owner = owner_d.cpu().numpy()
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        whole = core.count_device(up_d, it_d)
        torch.cuda.current_stream().synchronize()
        w = _Rows(whole, M)
        want = {a: w.row(a) for a in range(0, M, 997)}
        want.update({a: w.row(a) for a in range(0, 64)})
        w_nnz, w_rowsum = w.nnz.copy(), w.rowsum.copy()
    nnz_total = 0
    for part in range(3):
        with pkg.CooccurrenceCore(n_items=M, device=0) as core:
            res = core.count_device_owned(up_d, it_d, owner_d, part, freq_d, int(len(it)))
            torch.cuda.current_stream().synchronize()
            r = _Rows(res, M)
            mine = owner == part
            assert np.array_equal(r.nnz[mine], w_nnz[mine])
            assert np.all(r.nnz[~mine] == 0)
            assert np.array_equal(r.rowsum[mine], w_rowsum[mine])
            nnz_total += res.nnz
            for a, (wc, wn) in want.items():
                if owner[a] == part:
                    gc, gn = r.row(a)
                    assert np.array_equal(gc, wc) and np.array_equal(gn, wn)
    assert nnz_total == whole.nnz


def test_c5_topk_c3_shape_vs_oracle(pkg, oracle, torch_cuda):
    """C5 (LLR + top-50) on the large-universe path: the first 1,500 users of the C3 log, sampled rows'
    heaps against the oracle's rescorer (ItemRowRescorer...java:195-241), tolerance 1e-6 relative."""
    from tests._helpers import assert_row_topk, oracle_row_topk
    from flink_cooccurrence_amd import datagen

    up, it = datagen.c3_users(0, 1500)
    M, k = datagen.C3_ITEMS, 50
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        got = core.count(up, it)
        rs32 = got.rowsum32.astype(np.int64)
        observed = int(rs32.sum())
        rows = np.flatnonzero(np.diff(got.row_ptr))
        rng = np.random.default_rng(9)
        sample = np.unique(np.concatenate([rows[:6], rng.choice(rows, 40, replace=False)]))
        sizes, vals, scores = core.topk_items(sample, k)
        empty = np.setdiff1d(np.arange(0, M, 9973), rows)[:5]
        esz, _, _ = core.topk_items(empty, k)
        order = core.column_order()  # the device rows' column order (hot items first): the tie order
    assert np.all(esz == 0)
    for i, a in enumerate(sample.tolist()):
        s, e = got.row_ptr[a], got.row_ptr[a + 1]
        want = oracle_row_topk(oracle, got.cols[s:e], got.cnt16[s:e], rs32, a, k, observed, order)
        assert_row_topk(sizes[i], vals[i], scores[i], want, where=f"row {a}")


def test_c5_topk_owned_parts_vs_whole(pkg, torch_cuda):
    """Multi-GPU C5 on one GPU: 3 owned parts, each scored with the summed (all-reduced) row sums
    through cooc_topk_batch_device, equal the unpartitioned top-k on every owned row (bit for bit:
    same scores, same heap); rows owned elsewhere have size 0."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen, sharding

    up, it = datagen.c3_users(0, 3000)
    M, k = datagen.C3_ITEMS, 50
    dev = torch.device("cuda")
    up_d, it_d = torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev)
    freq_d = torch.from_numpy(np.bincount(it, minlength=M).astype(np.int64)).to(dev)
    owner_d = sharding.snake_owner(freq_d, 3)
    owner = owner_d.cpu().numpy()

    def topk(core, rowsum=None):
        sz = torch.empty(M, dtype=torch.int32, device=dev)
        v = torch.empty((M, k), dtype=torch.int32, device=dev)
        sc = torch.empty((M, k), dtype=torch.float64, device=dev)
        core.topk_batch_device(k, sz, v, sc, rowsum_global=rowsum)
        return sz.cpu().numpy(), v.cpu().numpy(), sc.cpu().numpy()

    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        core.count_device(up_d, it_d)
        w_sz, w_v, w_sc = topk(core)
    parts, rowsum = [], torch.zeros(M, dtype=torch.int64, device=dev)
    for part in range(3):
        core = pkg.CooccurrenceCore(n_items=M, device=0)
        core.count_device_owned(up_d, it_d, owner_d, part, freq_d, int(len(it)))
        rs = torch.empty(M, dtype=torch.int64, device=dev)
        core.copy_rowsum_device(rs)
        rowsum += rs
        parts.append(core)
    for part, core in enumerate(parts):
        sz, v, sc = topk(core, rowsum)
        mine = owner == part
        assert np.all(sz[~mine] == 0)
        assert np.array_equal(sz[mine], w_sz[mine])
        rows = np.flatnonzero(mine & (w_sz > 0))
        for a in rows[:: max(1, len(rows) // 2000)].tolist():
            n = int(w_sz[a])
            assert np.array_equal(v[a, :n], w_v[a, :n]) and np.array_equal(sc[a, :n], w_sc[a, :n], equal_nan=True), f"row {a}"
        core.close()


def test_underestimated_row_table_overflow_retries(pkg, torch_cuda):
    """A row whose partners are far more diverse than the global item frequencies predict: the planner
    sizes its hash chunk from the estimate, the LDS table overflows, and k_sp_main hands the whole row to
    the sort + segmented-reduce path (packed 64-bit (row, column) keys, radix sort, run counts: the north
    star's overflow fallback).  The path must have run, and the rows must be exact."""
    torch = torch_cuda
    rng = np.random.default_rng(21)
    M = 300_000
    lists = [rng.integers(8192, 8202, 10) for _ in range(10_000)]          # global mass on 10 columns
    for _ in range(3):                                                      # row 5: ~7,500 distinct partners
        lists.append(np.concatenate([[5], rng.choice(np.arange(20_000, M), 2500, replace=False), [7, 7]]))
    up = np.concatenate([[0], np.cumsum([len(x) for x in lists])]).astype(np.int64)
    it = np.concatenate(lists).astype(np.int32)
    dev = torch.device("cuda")
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        res = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
        torch.cuda.current_stream().synchronize()
        lens = np.diff(up)
        assert res.observed == int(np.sum(lens * (lens - 1)))
        n_sorted, pairs_sorted = core.last_sort_rows()
        assert n_sorted >= 1 and pairs_sorted >= 3 * 2500, (n_sorted, pairs_sorted)
        rows = _Rows(res, M)
        assert int(rows.rowsum.sum()) == res.observed
        _check_rows(rows, _Brute(up, it, M), [5, 7, 8192, 8195, 8201] + list(np.unique(it[it >= 20_000])[:20]))


@pytest.mark.parametrize("lens", [[], [0, 0, 0], [1, 0, 1, 1], [0, 2, 0, 3, 1, 0]])
def test_large_universe_empty_and_ragged(pkg, oracle, torch_cuda, lens):
    """Edge cases on the large-universe path (n_items = 100,000): no users, only empty users, users with
    single items (no pairs), ragged lists with repeats; against the closed form."""
    torch = torch_cuda
    M = 100_000
    rng = np.random.default_rng(len(lens))
    up = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    it = rng.choice([0, 1, 7, 40_000, M - 1], int(up[-1])).astype(np.int32)
    dev = torch.device("cuda")
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        res = core.count_device(torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev))
        torch.cuda.current_stream().synchronize()
        got = core.copy_batch(res.nnz, res.observed)
    rp, cols, data, rowsums, observed = oracle.closed_form(up, it, M)
    assert got.observed == observed and res.nnz == len(cols)
    assert np.array_equal(got.row_ptr, rp) and np.array_equal(got.cols, cols)
    assert np.array_equal(got.cnt.astype(np.int64), data) and np.array_equal(got.rowsum, rowsums)


def test_item_counts_vs_bincount(pkg, torch_cuda):
    """cooc_item_counts (the multi-GPU owner map's frequencies): equal to numpy's bincount on a C3-shaped
    log, LDS-counted hot ids and globally counted tail ids alike; ids outside [0, n_items) not counted."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    up, it = datagen.c3_users(0, 20_000)
    M = datagen.C3_ITEMS
    it_bad = np.concatenate([it, np.array([-1, M, M + 5], np.int32)])
    dev = torch.device("cuda")
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        got = core.item_counts(torch.from_numpy(it_bad).to(dev)).cpu().numpy()
        empty = core.item_counts(torch.zeros(0, dtype=torch.int32, device=dev)).cpu().numpy()
    assert np.array_equal(got, np.bincount(it, minlength=M))
    assert not empty.any()


@pytest.mark.parametrize("M", [40_500, 1_000_000])
def test_streaming_sparse_global_rows_vs_oracle(pkg, oracle, torch_cuda, M):
    """Streaming windows above the batch planner's range: the global rows are sorted row slabs merged
    per window (the rescorer's itemRows) instead of the dense matrix.  A window's delta rows come from one
    pass of the large-universe planner over its active users (old / new positions: a new position walks
    the user's whole history, an old one the window's new items, k_sp_window_contribs).  Every window's
    delta rows, row sums, observed and top-k against the oracle's rescorer, then the final global rows,
    row sums and accumulators; the slabs move and the arena compacts along the way."""
    from flink_cooccurrence_amd import datagen
    from tests._helpers import INT64_MAX, assert_windows_equal

    d = datagen.config_c1(seed=5, U=1500, M=M, mean=20.0)
    users, items, ts = datagen.to_records(d["user_ptr"], d["items"], d["ts"])
    op = pkg.NonSampledUserInteractionCounterOneInputStreamOperator(1, "SECONDS", n_items=M, top_k=10)
    ref = oracle.OracleStream(1000, topk=10)
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
    assert len(got) == len(want) > 5
    for g, w in zip(got, want):
        assert_windows_equal(g, w)
    assert op.accumulators() == ref.counters()
    rows, rp, cols, exact, v16 = ref.global_rows()
    for r in list(range(0, len(rows), max(1, len(rows) // 200))) + [len(rows) - 1]:
        a = int(rows[r])
        c, n, n16 = op.core.global_row(a)
        assert np.array_equal(c, cols[rp[r]:rp[r + 1]]), f"global row {a}"
        assert np.array_equal(n.astype(np.int64), exact[rp[r]:rp[r + 1]])
        assert np.array_equal(n16, v16[rp[r]:rp[r + 1]])
    gi, gv32, gex = ref.global_rowsums()
    ex, v32 = op.core.global_rowsums()
    assert np.array_equal(ex[gi], gex) and np.array_equal(v32[gi], gv32)
    op.close()


def test_c5_topk_long_rows_vs_oracle(pkg, oracle, torch_cuda):
    """Rows of tens of thousands of entries (88 chunks of 512 for one wave).  Two hubs: item 0 with
    45,000 partners of near-equal counts (ties everywhere: an entry equal to the heap's least must not
    enter, as in the sequential loop), and item 1 whose partners' counts grow with the column (later
    entries keep replacing the heap's least).  Both heaps, and short rows, against the oracle's
    rescorer (ItemRowRescorer...java:195-241), through the whole-batch launch and the sampled-rows
    launch."""
    torch = torch_cuda
    from tests._helpers import assert_row_topk, oracle_row_topk

    M, k = 50_000, 50
    rng = np.random.default_rng(31)
    users = []
    for b in range(2, 45_002):
        users.append([0, b])
        if b % 997 == 0:
            users.append([0, b])  # a few partners of hub 0 with count 2
    for b in range(2, 40_002, 1):
        for _ in range(1 + (b - 2) // 8_000):
            users.append([1, b])  # hub 1: counts 1..5 rising with the column
    for _ in range(20_000):
        users.append(sorted(rng.choice(np.arange(2, M), 3, replace=False).tolist()))
    lens = np.array([len(u) for u in users], np.int64)
    up = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    it = np.concatenate([np.array(u, np.int32) for u in users])
    dev = torch.device("cuda")
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        got = core.count(up, it)
        rs32 = got.rowsum32.astype(np.int64)
        observed = int(rs32.sum())
        assert got.row_ptr[1] - got.row_ptr[0] >= 45_000 and got.row_ptr[2] - got.row_ptr[1] >= 40_000
        sz = torch.empty(M, dtype=torch.int32, device=dev)
        v = torch.empty((M, k), dtype=torch.int32, device=dev)
        sc = torch.empty((M, k), dtype=torch.float64, device=dev)
        core.topk_batch_device(k, sz, v, sc)
        sz, v, sc = sz.cpu().numpy(), v.cpu().numpy(), sc.cpu().numpy()
        sample = np.array([0, 1, 2, 500, 20_001, 44_999], np.int64)
        s_sz, s_v, s_sc = core.topk_items(sample, k)
        order = core.column_order()
    for i, a in enumerate(sample.tolist()):
        s, e = got.row_ptr[a], got.row_ptr[a + 1]
        want = oracle_row_topk(oracle, got.cols[s:e], got.cnt16[s:e], rs32, a, k, observed, order)
        assert_row_topk(sz[a], v[a], sc[a], want, where=f"batch row {a}")
        assert_row_topk(s_sz[i], s_v[i], s_sc[i], want, where=f"sampled row {a}")
        n = int(sz[a])
        assert np.array_equal(v[a, :n], s_v[i, :n]) and np.array_equal(sc[a, :n], s_sc[i, :n], equal_nan=True)
