"""Shared test helpers: golden micro-logs, window comparison (oracle vs HIP path)."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INT64_MAX = (1 << 63) - 1


def micro_logs():
    with open(os.path.join(GOLDEN, "micro_logs.json")) as f:
        return json.load(f)["logs"]


def micro_events(log):
    """-> list of ('e', user, item, ts) / ('w', watermark) in arrival order."""
    if "events" in log:
        return [tuple(e) for e in log["events"]]
    g = log["generator"]
    ev = []
    if g["kind"] == "pairs":
        for u in range(g["users"]):
            for it in g["items"]:
                ev.append(("e", u, it, 500))
    elif g["kind"] == "repeat":
        for u in range(g["users"]):
            ev.extend([("e", u, g["item"], 500)] * g["times"])
    ev.append(("w", INT64_MAX))
    return ev


def micro_csr(log):
    """One-window micro-log -> (user_ptr, items) CSR in arrival order."""
    by_user: dict[int, list[int]] = {}
    for e in micro_events(log):
        if e[0] == "e":
            by_user.setdefault(e[1], []).append(e[2])
    users = sorted(by_user)
    lens = [len(by_user[u]) for u in users]
    user_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    items = np.array([i for u in users for i in by_user[u]], np.int32)
    return user_ptr, items


def run_events(events, process_element, process_watermark, batch=True):
    """Feed events to an operator; returns the list of fired windows."""
    out = []
    pend = []

    def flush():
        if pend:
            u, i, t = zip(*pend)
            process_element(np.array(u, np.int32), np.array(i, np.int32), np.array(t, np.int64))
            pend.clear()

    for e in events:
        if e[0] == "e":
            pend.append(e[1:])
        else:
            flush()
            out.extend(process_watermark(e[1]))
    flush()
    return out


def window_rows(w) -> dict:
    """{row: {col: exact}} of a fired window (oracle.WindowOutput or core.WindowResult)."""
    rows = {}
    for r, a in enumerate(w.rows.tolist()):
        s, e = int(w.row_ptr[r]), int(w.row_ptr[r + 1])
        rows[a] = dict(zip(w.cols[s:e].tolist(), w.exact[s:e].tolist()))
    return rows


def window_rows16(w) -> dict:
    rows = {}
    for r, a in enumerate(w.rows.tolist()):
        s, e = int(w.row_ptr[r]), int(w.row_ptr[r + 1])
        rows[a] = dict(zip(w.cols[s:e].tolist(), w.v16[s:e].tolist()))
    return rows


def as_int_keys(d):
    return {int(k): (as_int_keys(v) if isinstance(v, dict) else v) for k, v in d.items()}


def assert_windows_equal(got, want, topk_rtol=1e-6):
    """Bit-exact delta rows / row sums / observed; top-k by the tolerance contract of SURVEY §8(a)."""
    assert got.ts == want.ts
    assert np.array_equal(got.rows, want.rows), "delta row set differs"
    assert np.array_equal(got.row_ptr, want.row_ptr), "delta row lengths differ"
    assert np.array_equal(got.cols, want.cols), "delta columns differ"
    assert np.array_equal(np.asarray(got.exact, np.int64), np.asarray(want.exact, np.int64)), "exact counts differ"
    assert np.array_equal(got.v16, want.v16), "int16 view differs"
    assert np.array_equal(got.rs_items, want.rs_items)
    assert np.array_equal(got.rs_exact, want.rs_exact)
    assert np.array_equal(got.rs_v32, want.rs_v32)
    assert got.observed == want.observed
    if len(want.topk_rows) or len(got.topk_rows):
        assert_topk_equal(got, want, topk_rtol)


def assert_topk_equal(got, want, rtol=1e-6):
    assert np.array_equal(got.topk_rows, want.topk_rows)
    assert np.array_equal(got.topk_sizes, want.topk_sizes)
    for r in range(len(want.topk_rows)):
        n = int(want.topk_sizes[r])
        gs, ws = got.topk_scores[r, :n], want.topk_scores[r, :n]
        gv, wv = got.topk_values[r, :n], want.topk_values[r, :n]
        # The heap layouts agree exactly whenever every score agrees bit for bit (same iteration
        # order, same comparisons).  Scores may differ by a few ulp (device vs glibc log), so compare
        # the score multisets with a tolerance and the item sets strictly above the k-th score.
        nan_g, nan_w = np.isnan(gs), np.isnan(ws)
        assert np.array_equal(np.sort(nan_g), np.sort(nan_w)), "NaN scores differ"
        g_sorted = np.sort(gs[~nan_g])
        w_sorted = np.sort(ws[~nan_w])
        tol = np.maximum(rtol * np.abs(w_sorted), 1e-9)
        assert np.all(np.abs(g_sorted - w_sorted) <= tol), f"row {want.topk_rows[r]}: scores differ"
        if n and not nan_w.any():
            kth = w_sorted[0]
            margin = max(rtol * abs(kth), 1e-9)
            assert set(gv[gs > kth + margin].tolist()) == set(wv[ws > kth + margin].tolist())


def oracle_row_topk(oracle, cols, cnt16, rs32, a: int, k: int, observed: int, order=None):
    """The rescorer's heap for row a (ItemRowRescorer...java:195-223) fed in the device's column order --
    ascending order[col] (CooccurrenceCore.column_order(); None: ascending column id) -- with the
    reference's views: int16 counts, int32 row sums, observed = sum of the int32 row sums."""
    q = oracle.PriorityQueue(k)
    cols, cnt16 = np.asarray(cols), np.asarray(cnt16)
    if order is not None:
        o = np.argsort(np.asarray(order)[cols], kind="stable")
        cols, cnt16 = cols[o], cnt16[o]
    for b, c16 in zip(cols.tolist(), cnt16.tolist()):
        sc = oracle.score_item(int(c16), int(rs32[a]), int(rs32[b]), observed)
        if q.size() < k:
            q.add(b, sc)
        elif sc > q.least_score():
            q.update(b, sc)
    return q.entries()


def llr_atol(observed: int) -> float:
    """SURVEY.md §8(a)'s cancellation bound for one LLR score: 64 ulp of the largest x log x term,
    xLogX(k11 + k12 + k21 + k22) = xLogX(observed + 2 k11) (ItemRowRescorer...java:238), with k11 at most
    the int16 range.  A 1-ulp difference of that term between two log implementations moves a score by
    ~ulp(x log x) absolutely, which is above 1e-6 relative for the weak scores of a large log."""
    x = abs(int(observed)) + 2 * 32768
    return 64 * np.finfo(np.float64).eps * x * np.log(max(x, 2))


def assert_row_topk(size, vals, scores, want, rtol=1e-6, where="", atol=1e-9):
    """One row's heap against the oracle's: scores within max(rtol |ref|, atol) (NaN where NaN); the identical
    heap layout when every score agrees bit for bit; otherwise (a score a few ulp off can move an item within
    the heap, or swap two near-equal items at the boundary) the items whose scores lie clearly above the k-th
    score -- more than the tolerance above it -- are the same set (SURVEY.md §8(a) parity item 4).
    Returns True when the heap matched bit for bit (layout and scores)."""
    assert int(size) == len(want), f"{where}: heap size {size} != {len(want)}"
    wv = np.array([v for v, _ in want], np.int32)
    ws = np.array([x for _, x in want], np.float64)
    gs = np.asarray(scores[: int(size)], np.float64)
    gv = np.asarray(vals[: int(size)])
    assert np.array_equal(np.isnan(gs), np.isnan(ws)), f"{where}: NaN scores differ"
    fin = ~np.isnan(ws)
    tol = np.maximum(rtol * np.abs(ws[fin]), atol)
    assert np.all(np.abs(gs[fin] - ws[fin]) <= tol), (
        f"{where}: scores differ by up to {np.max(np.abs(gs[fin] - ws[fin])) if fin.any() else 0} (atol {atol})")
    if np.array_equal(gs[fin], ws[fin]):
        assert np.array_equal(gv, wv), f"{where}: heap layout differs"
        return True
    if fin.all() and len(ws):
        kth = float(np.min(ws))
        margin = 2 * float(np.max(tol))
        assert set(gv[gs > kth + margin].tolist()) == set(wv[ws > kth + margin].tolist()), (
            f"{where}: items above the k-th score differ")
    return False
