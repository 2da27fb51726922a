"""The job's text source (FlinkCooccurrences.java:55-61,207-229) through the C-ABI (host-only).

Semantics restated from the reference: TextInputFormat lines ('\\n', a trailing '\\r' dropped, a last
line without '\\n' kept), String.split(",") (fields after the third ignored), Integer.valueOf /
Long.valueOf (sign + decimal digits, range-checked, no spaces), AscendingTimestampExtractor
watermark = largest timestamp - 1.
"""
import numpy as np
import pytest

from tests._helpers import INT64_MAX


def test_parse_golden(pkg):
    data = (b"1,2,3\n"
            b"-5,+7,-9\r\n"                      # signs; "\r\n" line end
            b"2147483647,-2147483648,9223372036854775807\n"
            b"4,5,6,extra,fields\n"              # split()[3..] unused
            b"7,8,-9223372036854775808")         # last line without '\n'
    u, i, t = pkg.parse_interactions(data)
    assert u.tolist() == [1, -5, 2147483647, 4, 7]
    assert i.tolist() == [2, 7, -2147483648, 5, 8]
    assert t.tolist() == [3, -9, 2**63 - 1, 6, -2**63]
    assert pkg.parse_interactions(b"")[0].size == 0
    assert pkg.parse_interactions(b"1,2,3\n")[0].size == 1  # no record after the final '\n'


@pytest.mark.parametrize("bad,line", [
    (b"1,2,3\n\n4,5,6\n", 1),          # empty line: Integer.valueOf("")
    (b"1,2\n", 0),                     # split[2] out of bounds
    (b"1, 2,3\n", 0),                  # no whitespace in Integer.valueOf
    (b"2147483648,1,1\n", 0),          # int overflow
    (b"1,1,9223372036854775808\n", 0),  # long overflow
    (b"1,,3\n", 0),                    # empty middle field
    (b"1,2,3\n+,1,1\n", 1),            # a sign alone
    (b"1,2,0x10\n", 0),
])
def test_parse_rejects_like_the_splitter(pkg, bad, line):
    with pytest.raises(pkg.IllegalArgumentException, match=f"line {line} "):
        pkg.parse_interactions(bad)


def test_parse_round_trip_random(pkg):
    rng = np.random.default_rng(4)
    n = 20_000
    u = rng.integers(-2**31, 2**31, n, dtype=np.int64)
    i = rng.integers(0, 5000, n)
    t = np.sort(rng.integers(-2**62, 2**62, n, dtype=np.int64))
    text = "".join(f"{a},{b},{c}\n" for a, b, c in zip(u, i, t)).encode()
    pu, pi, pt = pkg.parse_interactions(text)
    assert np.array_equal(pu, u) and np.array_equal(pi, i) and np.array_equal(pt, t)


def test_text_source_drives_oracle_semantics(oracle):
    """The watermark rule of run_text_source (largest ts - 1 after every block, MAX at the end)
    applied to the oracle: every record is on time (ascending timestamps), all windows fire."""
    from flink_cooccurrence_amd import datagen

    d = datagen.config_c1(seed=1, U=200, M=50, mean=10.0)
    users, items, ts = datagen.to_records(d["user_ptr"], d["items"], d["ts"])
    s = oracle.OracleStream(1000)
    hi = None
    for lo in range(0, len(users), 500):
        sl = slice(lo, lo + 500)
        assert s.process_elements(users[sl], items[sl], ts[sl]) == 0
        hi = int(ts[sl].max()) if hi is None else max(hi, int(ts[sl].max()))
        s.process_watermark(hi - 1)
    s.process_watermark(INT64_MAX)
    assert s.counters()["UserInteractionCounterLateElements"] == 0
