"""Exactness of the large-universe path (k_sp_main, the C3 / C5 hot path) at the benchmark's sizes.

Every row of the device result is compared with an independent CPU restatement through per-row
fingerprints (cooc_verify_batch: checksum = sum over the row's keys of splitmix64(col << 32 ^ count),
key count, count sum; oracle.RowChecks restates the same):

* 1/256 of the C3 log (39,062 users, ~1e9 ordered pairs) against the record-by-record restatement
  (oracle.count_batch_mt_rows: NonSampled...java:129-161 records into Int2ShortOpenHashMap
  restatements, ItemRowAggregator.java:26-31), plus the symmetry of every entry;
* 1/64 (~4.2e9 pairs) and the benchmark's own workload, 1/8 of C3 (1.25e6 users, 3.36e10 pairs, what
  bench.py times), against the closed-form restatement (oracle.row_checksums; it agrees with the
  record-by-record one and with scipy in tests/test_oracle_semantics.py);
* the same log with its item ids permuted (datagen.c3_item_perm: ids carry no popularity order), at 1/256
  and at the benchmark's 1/8 (bench.py --permute-items).

Bar: bit-exact (every row's fingerprint, key count and count sum equal), plus the device-side
invariants (sum of counts == sum of row sums == P, sorted rows, no zero count).  Needs an MI355X.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _threads():
    from bench import cpu_threads

    return cpu_threads()[0]


def _device_checks(pkg, torch, up_d, it_d, M, symmetry, any_order=False):
    dev = up_d.device
    with pkg.CooccurrenceCore(n_items=M, device=dev.index or 0, any_order=any_order) as core:
        res = core.count_device(up_d, it_d)
        cs = torch.zeros(M, dtype=torch.int64, device=dev)
        chk = core.verify_batch(symmetry=symmetry, row_checksum=cs)
        torch.cuda.synchronize()
        nnz = np.zeros(M, np.int32)
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipMemcpy(nnz.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(res.row_nnz),
                             ctypes.c_size_t(nnz.nbytes), ctypes.c_int(2)) == 0
        return res, chk, cs.cpu().numpy().view(np.uint64), nnz


def _compare(res, chk, cs, nnz, want, P):
    assert res.observed == P == want.pairs
    assert chk["rows_bad_sum"] == 0 and chk["rows_bad_entries"] == 0
    assert chk["sum_counts"] == chk["sum_rowsums"] == P
    assert chk["entries"] == res.nnz == want.distinct
    assert np.array_equal(nnz.astype(np.int64), want.nnz), "per-row key counts differ"
    bad = np.flatnonzero(cs != want.checksum)
    assert len(bad) == 0, f"{len(bad)} rows differ from the oracle, e.g. {bad[:10].tolist()}"


@pytest.mark.parametrize("permute", [False, True])
def test_c3_256th_every_row_vs_record_by_record_oracle(pkg, oracle, torch_cuda, permute):
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    U, M = datagen.C3_USERS // 256, datagen.C3_ITEMS
    up, it = datagen.c3_users(0, U, permute=permute)
    dev = torch.device("cuda", 0)
    res, chk, cs, nnz = _device_checks(pkg, torch, torch.from_numpy(up).to(dev), torch.from_numpy(it).to(dev), M,
                                       symmetry=True)
    assert chk["asymmetric_entries"] == 0
    want = oracle.count_batch_mt_rows(up, it, M, _threads())
    _compare(res, chk, cs, nnz, want, datagen.ordered_pairs(up))


@pytest.mark.parametrize("share,permute,any_order", [(64, False, False), (8, False, False), (8, True, False),
                                                     (8, False, True), (64, True, True)])
def test_c3_share_every_row_vs_closed_form_oracle(pkg, oracle, torch_cuda, share, permute, any_order):
    """share = 8 is the benchmark's workload (bench.py, N = 1): users [0, 1.25e6) of the 1B log.  any_order:
    COOC_FLAG_ANY_ORDER (rows in no particular order; the fingerprints are order-independent sums)."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    U, M = datagen.C3_USERS // share, datagen.C3_ITEMS
    dev = torch.device("cuda", 0)
    up_d, it_d = datagen.c3_users(0, U, device=dev, permute=permute)
    res, chk, cs, nnz = _device_checks(pkg, torch, up_d, it_d, M, symmetry=share >= 64, any_order=any_order)
    if share >= 64 and not any_order:
        assert chk["asymmetric_entries"] == 0
    up, it = up_d.cpu().numpy(), it_d.cpu().numpy()
    del up_d, it_d
    want = oracle.row_checksums(up, it, M, _threads())
    _compare(res, chk, cs, nnz, want, datagen.c3_ordered_pairs(0, U))


def test_c3_64th_in_a_64_tile_universe(pkg, oracle, torch_cuda):
    """n_items = 1,040,000 (the top 40,000 ids unused): 64 column tiles, every bit of a row plan's 64-bit
    tile masks a tile -- the gather mode's flag lives outside them (it was bit 63 of the dense mask, which
    turned gather mode off for 64-tile universes: 1.6x slower).  1/64 of C3, bit-exact against the closed form."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    U, M = datagen.C3_USERS // 64, 1_040_000
    dev = torch.device("cuda", 0)
    up_d, it_d = datagen.c3_users(0, U, device=dev)
    res, chk, cs, nnz = _device_checks(pkg, torch, up_d, it_d, M, symmetry=True)
    assert chk["asymmetric_entries"] == 0
    up, it = up_d.cpu().numpy(), it_d.cpu().numpy()
    del up_d, it_d
    want = oracle.row_checksums(up, it, M, _threads())
    _compare(res, chk, cs, nnz, want, datagen.c3_ordered_pairs(0, U))


def _d2h(ptr, n, dtype, offset=0):
    import ctypes

    out = np.zeros(n, dtype)
    if n:
        hip = ctypes.CDLL("libamdhip64.so")
        src = ctypes.c_void_p(ptr + offset * out.itemsize)
        assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), src, ctypes.c_size_t(out.nbytes), ctypes.c_int(2)) == 0
    return out


def test_c5_topk_benched_share_vs_oracle(pkg, oracle, torch_cuda):
    """C5 at the benchmark's size (bench.py --config c5: 1/8 of C3, top-50, the reference's int16 / int32
    views): the device heaps of rows 0-63 (the hottest: ~1e6 entries, int16 wraps), 1,000 random rows and
    EVERY row whose heap root is NaN (a wrapped k11 < 0 or the reference's k22 = observed + k11 - k12 - k21
    going negative, ItemRowRescorer...java:238) against the oracle's rescorer loop (ItemRowRescorer...java:
    195-223, LogLikelihood.java:41-57, IntDoublePriorityQueue.java:132-205) fed each row's entries in the
    device row's order (the tie order).  Scores within SURVEY §8(a)'s bound max(1e-6 |ref|, 64 ulp of
    xLogX(observed + 2 k11)) (the LLR's cancellation: at observed ~ 3e10 one ulp of the log terms is ~1e-4),
    NaN where NaN; the identical heap layout whenever every score agrees bit for bit."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen

    from tests._helpers import assert_row_topk, llr_atol

    U, M, k = datagen.C3_USERS // 8, datagen.C3_ITEMS, 50
    dev = torch.device("cuda", 0)
    up_d, it_d = datagen.c3_users(0, U, device=dev)
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        res = core.count_device(up_d, it_d)
        del up_d, it_d
        sizes = torch.empty(M, dtype=torch.int32, device=dev)
        vals = torch.empty((M, k), dtype=torch.int32, device=dev)
        scores = torch.empty((M, k), dtype=torch.float64, device=dev)
        core.topk_batch_device(k, sizes, vals, scores)
        rowsum = torch.empty(M, dtype=torch.int64, device=dev)
        core.copy_rowsum_device(rowsum)
        torch.cuda.synchronize()
        sz, v, sc = sizes.cpu().numpy(), vals.cpu().numpy(), scores.cpu().numpy()
        del vals, scores
        rs = rowsum.cpu().numpy()
        base = _d2h(res.row_base, M, np.int64)
        nnz = _d2h(res.row_nnz, M, np.int32).astype(np.int64)
        rng = np.random.default_rng(42)
        nonempty = np.flatnonzero(nnz)
        nan_all = np.flatnonzero((sz > 0) & np.isnan(sc[:, 0]))
        # (nearly every heap of this share is NaN-rooted, and the oracle reads such a row whole: a sample of them)
        nan_root = np.sort(rng.choice(nan_all, min(len(nan_all), 20_000), replace=False))
        rows = np.unique(np.concatenate([np.arange(64), rng.choice(nonempty, 1000, replace=False), nan_root]))
        rp = np.concatenate([[0], np.cumsum(nnz[rows])])
        cols = np.zeros(int(rp[-1]), np.int32)
        cnt = np.zeros(int(rp[-1]), np.uint32)
        for j, a in enumerate(rows.tolist()):  # each row in the device's own order (the tie order)
            cols[rp[j]:rp[j + 1]] = _d2h(res.col, int(nnz[a]), np.int32, int(base[a]))
            cnt[rp[j]:rp[j + 1]] = _d2h(res.cnt, int(nnz[a]), np.uint32, int(base[a]))
    rs32 = rs.astype(np.int64).astype(np.uint64).astype(np.uint32).view(np.int32)  # Java int row sums
    observed = int(rs32.astype(np.int64).sum())  # the rescorer's long: the sum of the int deltas (:154)
    cnt16 = cnt.astype(np.uint16).view(np.int16)
    w_sz, w_v, w_sc = oracle.rows_topk(rows, rp, cols, cnt16, rs32, observed, k, _threads())
    assert len(nan_root) > 0, "the benched share has NaN heap roots (int16 wraps): they must be covered"
    atol = llr_atol(observed)
    worst = 0.0
    exact = 0
    for j, a in enumerate(rows.tolist()):
        want = [(int(w_v[j, i]), float(w_sc[j, i])) for i in range(int(w_sz[j]))]
        exact += assert_row_topk(sz[a], v[a], sc[a], want, where=f"row {a}", atol=atol)
        fin = ~np.isnan(w_sc[j, :w_sz[j]])
        if fin.any():
            worst = max(worst, float(np.max(np.abs(sc[a, :w_sz[j]][fin] - w_sc[j, :w_sz[j]][fin]))))
    print(f"largest score difference {worst:.3g} (bound {atol:.3g})")
    print(f"checked {len(rows)} heaps ({len(nan_root)} of the {len(nan_all)} with a NaN root) over {int(rp[-1])} entries; "
          f"{exact} ({exact / len(rows):.1%}) identical bit for bit (layout and every score)")
    # (kept where a GPU run collects its outputs, gpurun_out/, so the match rate survives a -q log)
    import json
    import os

    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "c5_heap_match.json"), "w") as f:
            json.dump({"heaps_checked": len(rows), "nan_root_heaps": len(nan_all), "nan_root_heaps_checked": len(nan_root),
                       "entries": int(rp[-1]),
                       "bit_identical": exact, "bit_identical_frac": exact / len(rows),
                       "largest_score_difference": worst, "bound": atol}, f, indent=1)
    # both sides take their logs from Java's StrictMath.log (fdlibm): every heap matches bit for bit
    assert exact == len(rows), f"only {exact} of {len(rows)} heaps match bit for bit"


def test_c5_owner_unit_vs_oracle(pkg, oracle, torch_cuda):
    """C5 in the regime C5 runs in (bench.py --config c5 at N = 1): one rank's unit of the 8-GPU job -- the whole 1B
    log resident, the rows rank 0 owns counted over every user, scored against the WHOLE log's row sums and observed
    total (the all-reduced row sums), top-50 in the reference's int16 / int32 views.  Checked against the oracle's
    rescorer loop (ItemRowRescorer...java:195-223, LogLikelihood.java:41-57, IntDoublePriorityQueue.java:132-205)
    fed each row's entries in the device row's order (the tie order): at least 1,000 heaps whose root is a number
    (the top-k selection with the `score > least` replacement of :218-222 at work), the owned rows among the 64
    hottest, and every NaN-rooted heap.  Both sides take their logs from Java's StrictMath.log (fdlibm), so every
    heap must match bit for bit: layout, values and scores."""
    torch = torch_cuda
    from flink_cooccurrence_amd import datagen, sharding

    from tests._helpers import assert_row_topk

    M, k, world, part = datagen.C3_ITEMS, 50, 8, 0
    dev = torch.device("cuda", 0)
    up_d, it_d = datagen.c3_log_device(dev)
    with pkg.CooccurrenceCore(n_items=M, device=0) as core:
        freq = core.item_counts(it_d)
        owner = sharding.snake_owner(freq, world)
        rs_g = datagen.closed_form_rowsums_device(up_d, it_d, M)
        res = core.count_device_owned(up_d, it_d, owner, part, freq, int(it_d.numel()))
        del up_d, it_d
        sizes = torch.empty(M, dtype=torch.int32, device=dev)
        vals = torch.empty((M, k), dtype=torch.int32, device=dev)
        scores = torch.empty((M, k), dtype=torch.float64, device=dev)
        core.topk_batch_device(k, sizes, vals, scores, rowsum_global=rs_g)
        torch.cuda.synchronize()
        sz, v, sc = sizes.cpu().numpy(), vals.cpu().numpy(), scores.cpu().numpy()
        own = (owner == part).cpu().numpy()
        rs = rs_g.cpu().numpy()
        del vals, scores, rs_g
        base = _d2h(res.row_base, M, np.int64)
        nnz = _d2h(res.row_nnz, M, np.int32).astype(np.int64)
        assert np.array_equal(nnz > 0, own & (rs > 0)), "rows outside the owned part must be empty"
        rng = np.random.default_rng(43)
        filled = np.flatnonzero(sz > 0)
        nan_root = filled[np.isnan(sc[filled, 0])]
        num_root = filled[~np.isnan(sc[filled, 0])]
        hot = np.flatnonzero(own[:64] & (nnz[:64] > 0))
        rows = np.unique(np.concatenate([hot, rng.choice(num_root, 1200, replace=False), nan_root]))
        rp = np.concatenate([[0], np.cumsum(nnz[rows])])
        cols = np.zeros(int(rp[-1]), np.int32)
        cnt = np.zeros(int(rp[-1]), np.uint32)
        for j, a in enumerate(rows.tolist()):  # each row in the device's own order (the tie order)
            cols[rp[j]:rp[j + 1]] = _d2h(res.col, int(nnz[a]), np.int32, int(base[a]))
            cnt[rp[j]:rp[j + 1]] = _d2h(res.cnt, int(nnz[a]), np.uint32, int(base[a]))
    rs32 = rs.astype(np.int64).astype(np.uint64).astype(np.uint32).view(np.int32)  # Java int row sums
    observed = int(rs32.astype(np.int64).sum())  # the rescorer's long: the sum of the int deltas (:154)
    cnt16 = cnt.astype(np.uint16).view(np.int16)
    w_sz, w_v, w_sc = oracle.rows_topk(rows, rp, cols, cnt16, rs32, observed, k, _threads())
    exact = 0
    n_num = 0
    for j, a in enumerate(rows.tolist()):
        want = [(int(w_v[j, i]), float(w_sc[j, i])) for i in range(int(w_sz[j]))]
        exact += assert_row_topk(sz[a], v[a], sc[a], want, where=f"row {a}", atol=0.0)
        n_num += int(w_sz[j] > 0 and not np.isnan(w_sc[j, 0]))
    frac_nan = len(nan_root) / max(len(filled), 1)
    print(f"owned heaps {len(filled)}, NaN-rooted {len(nan_root)} ({frac_nan:.2%}); checked {len(rows)} heaps "
          f"({n_num} with a numeric root, {len(hot)} of the 64 hottest rows) over {int(rp[-1])} entries; {exact} "
          f"identical bit for bit")
    import json
    import os

    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "c5_owner_heap_match.json"), "w") as f:
            json.dump({"unit": f"rank {part} of {world}: whole 1B log, owned rows, whole-log row sums",
                       "owned_heaps": len(filled), "nan_root_heaps": len(nan_root), "nan_root_frac": frac_nan,
                       "heaps_checked": len(rows), "numeric_root_heaps_checked": n_num, "entries": int(rp[-1]),
                       "bit_identical": exact}, f, indent=1)
    assert n_num >= 1000
    assert exact == len(rows), f"only {exact} of {len(rows)} heaps match bit for bit"
