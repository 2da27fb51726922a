"""The ItemCooccurrences wire codec (ItemCooccurrences.java:113-147) through the C-ABI (host-only
entry points: no GPU needed).

Pinning: Kryo is a Maven dependency of Flink 1.3.2 (Kryo 2.24.0), not vendored, and no serialized
ItemCooccurrences bytes ship with the reference, so the byte vectors below are derived by hand from
Kryo's published primitives (Output.writeVarInt(v, true): 7-bit groups, least significant first,
bit 7 = more, <= 5 bytes; Output.writeShort: high byte first).  "parity unpinned" by reference
fixtures; pinned by the derivations and by a semantic round trip against the oracle.
"""
import numpy as np
import pytest

from tests._helpers import INT64_MAX

# (items, increments, rec_ptr, others, ks) -> bytes, each derived by hand
VECTORS = [
    # item 5, inc +1, size 2, others [3, 4]:  05 | 00 01 | 02 | 03 04
    (([5], [1], [0, 2], [3, 4], None), bytes([0x05, 0x00, 0x01, 0x02, 0x03, 0x04])),
    # item 300 = 0b10_0101100 -> AC 02; inc -1 -> FF FF; size 1; other 127 -> 7F
    (([300], [-1], [0, 1], [127], None), bytes([0xAC, 0x02, 0xFF, 0xFF, 0x01, 0x7F])),
    # other 128 -> 80 01; other 16384 -> 80 80 01
    (([0], [1], [0, 2], [128, 16384], None), bytes([0x00, 0x00, 0x01, 0x02, 0x80, 0x01, 0x80, 0x80, 0x01])),
    # a negative int takes 5 bytes with optimizePositive: -1 -> FF FF FF FF 0F
    (([-1], [256], [0, 0], [], None), bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x0F, 0x01, 0x00, 0x00])),
    # k = 1 skips slot 1 and writes size - 1 (:124-131): [7, 8, 9] -> 2 | 07 09
    (([2], [1], [0, 3], [7, 8, 9], [1]), bytes([0x02, 0x00, 0x01, 0x02, 0x07, 0x09])),
    # Integer.MAX_VALUE -> FF FF FF FF 07; two records back to back
    (([2**31 - 1, 1], [1, 1], [0, 0, 1], [6], None),
     bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x07, 0x00, 0x01, 0x00, 0x01, 0x00, 0x01, 0x01, 0x06])),
]


@pytest.mark.parametrize("i", range(len(VECTORS)))
def test_encode_golden(pkg, i):
    (items, incs, rp, others, ks), want = VECTORS[i]
    assert pkg.encode_item_cooccurrences(items, incs, rp, others, ks) == want


@pytest.mark.parametrize("i", range(len(VECTORS)))
def test_decode_golden(pkg, i):
    (items, incs, rp, others, ks), data = VECTORS[i]
    it, inc, rp2, ot = pkg.decode_item_cooccurrences(data)
    if ks is not None:  # the reader always sees k == -1 (:144): slot k is gone
        keep = [j for r in range(len(items)) for j in range(rp[r], rp[r + 1]) if j - rp[r] != ks[r]]
        others = [others[j] for j in keep]
        rp = [0] + list(np.cumsum([rp[r + 1] - rp[r] - 1 for r in range(len(items))]))
    assert it.tolist() == items and inc.tolist() == incs and rp2.tolist() == list(rp) and ot.tolist() == others


def test_round_trip_random(pkg):
    rng = np.random.default_rng(3)
    n = 500
    lens = rng.integers(0, 40, n)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    others = rng.integers(-2**31, 2**31, rp[-1], dtype=np.int64).astype(np.int32)
    others[::3] = rng.integers(0, 1000, len(others[::3]))
    items = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    incs = rng.integers(-2**15, 2**15, n).astype(np.int16)
    data = pkg.encode_item_cooccurrences(items, incs, rp, others)
    it, inc, rp2, ot = pkg.decode_item_cooccurrences(data)
    assert np.array_equal(it, items) and np.array_equal(inc, incs)
    assert np.array_equal(rp2, rp) and np.array_equal(ot, others)
    assert pkg.decode_item_cooccurrences(b"")[0].size == 0


@pytest.mark.parametrize("bad", [bytes([0x05]), bytes([0x05, 0x00]), bytes([0x05, 0x00, 0x01, 0x02, 0x03]),
                                 bytes([0x05, 0x00, 0x01, 0x80]),
                                 bytes([0x05, 0x00, 0x01, 0xFF, 0xFF, 0xFF, 0xFF, 0x0F])])  # size -1
def test_decode_malformed_is_illegal_argument(pkg, bad):
    with pytest.raises(pkg.IllegalArgumentException):
        pkg.decode_item_cooccurrences(bad)


def test_encode_bad_k(pkg):
    with pytest.raises(pkg.IllegalArgumentException):
        pkg.encode_item_cooccurrences([1], [1], [0, 2], [3, 4], [2])


def test_emitted_records_reduce_to_window_rows(pkg, oracle):
    """Emit the records NonSampled...java:138-151 sends for one window (item, history, +1) and
    (other, [item], +1), encode them, decode them, reduce them by key as ItemRowAggregator.add does
    (:26-31): the oracle's window delta rows."""
    rng = np.random.default_rng(8)
    U, M = 25, 30
    hist = [rng.integers(0, M, rng.integers(1, 9)).tolist() for _ in range(U)]
    items, incs, others, rp = [], [], [], [0]
    for h in hist:
        for q, x in enumerate(h):
            if q == 0:
                continue
            items.append(x); incs.append(1); others += h[:q]; rp.append(len(others))  # :138-139
            for o in h[:q]:
                items.append(o); incs.append(1); others.append(x); rp.append(len(others))  # :144-147
    it, inc, rp2, ot = pkg.decode_item_cooccurrences(pkg.encode_item_cooccurrences(items, incs, rp, others))
    red = {}
    for r in range(len(it)):
        for o in ot[rp2[r]:rp2[r + 1]]:
            red[(int(it[r]), int(o))] = red.get((int(it[r]), int(o)), 0) + int(inc[r])
    users = np.concatenate([[u] * len(h) for u, h in enumerate(hist)]).astype(np.int32)
    flat = np.concatenate(hist).astype(np.int32)
    s = oracle.OracleStream(1000)
    s.process_elements(users, flat, np.zeros(len(flat), np.int64))
    (w,) = s.process_watermark(INT64_MAX)
    want = {(int(a), int(b)): int(v) for r, a in enumerate(w.rows)
            for b, v in zip(w.cols[w.row_ptr[r]:w.row_ptr[r + 1]], w.exact[w.row_ptr[r]:w.row_ptr[r + 1]])}
    assert red == want
