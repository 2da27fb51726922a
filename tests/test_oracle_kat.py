"""The oracle against the reference's own known-answer tests (CPU).

LogLikelihoodTest.java:11-17 and IntDoublePriorityQueueTest.java:12-98 restated against the C
restatement of LogLikelihood / IntDoublePriorityQueue.  java.util.Random is restated to regenerate
IntDoublePriorityQueueTest's inputs; its own pin is the widely published first outputs of
`new Random(42)` (nextInt() = -1170105035, nextDouble() = 0.7275636800328681).
"""
import numpy as np
import pytest


def test_log_likelihood_ratio_kat(oracle):
    # LogLikelihoodTest.java:14-16, tolerance 0.1 as in the reference
    assert oracle.llr(110, 2442, 111, 29114) == pytest.approx(270.72, abs=0.1)
    assert oracle.llr(29, 13, 123, 31612) == pytest.approx(263.90, abs=0.1)
    assert oracle.llr(9, 12, 429, 31327) == pytest.approx(48.94, abs=0.1)


def test_llr_round_off_clamp_and_zero_cells(oracle):
    # LogLikelihood.java:51-53: row + column < matrix -> 0.0; xLogX(0) = 0 (:59-61)
    assert oracle.llr(0, 0, 0, 0) == 0.0
    assert oracle.llr(1, 0, 0, 0) == 0.0
    assert oracle.llr(5, 0, 0, 5) > 0.0


def test_score_item_nonstandard_k22(oracle):
    # ItemRowRescorer...java:236-240: k22 = observed + k11 - k12 - k21 (not N - k11 - k12 - k21)
    k11, rs_a, rs_b, obs = 3, 10, 12, 100
    k12, k21 = rs_a - k11, rs_b - k11
    assert oracle.score_item(k11, rs_a, rs_b, obs) == oracle.llr(k11, k12, k21, obs + k11 - k12 - k21)


def test_negative_short_count_is_nan(oracle):
    # a wrapped (short) count makes a cell negative: Math.log(negative) = NaN propagates
    assert np.isnan(oracle.score_item(-32768, 32768, 32768, 65536))


def test_java_random_pins(oracle):
    assert oracle.java_random_next_int32(42, 1)[0] == -1170105035
    assert oracle.java_random_doubles(42, 1)[0] == 0.7275636800328681


def test_pq_add_ascending_order(oracle):  # IntDoublePriorityQueueTest.java:12-22
    q = oracle.PriorityQueue(10)
    for i in range(10):
        q.add(i, float(i))
    assert q.least_value() == 0 and q.least_score() == 0.0


def test_pq_add_descending_order(oracle):  # :24-34
    q = oracle.PriorityQueue(10)
    for i in range(9, -1, -1):
        q.add(i, float(i))
    assert q.least_value() == 0 and q.least_score() == 0.0


def test_pq_random_elements(oracle):  # :36-75
    scores = oracle.java_random_doubles(0xC0FFEE, 100)
    q = oracle.PriorityQueue(10)
    for i in range(100):
        if q.size() < 10:
            q.add(i, scores[i])
        elif scores[i] > q.least_score():
            q.update(i, scores[i])
    s = np.sort(scores)
    assert q.least_score() == s[90]
    top = [sc for _, sc in q.entries()]
    assert top[0] == s[90]
    assert np.array_equal(np.sort(top), s[90:])


def test_pq_add_and_clear(oracle):  # :77-98
    q = oracle.PriorityQueue(10)
    q.add(0, 0.0)
    q.add(1, 1.0)
    q.add(2, 2.0)
    assert q.size() == 3
    q.reset()
    for i in range(10):
        q.add(i, float(i))
    assert q.size() == 10 and q.least_value() == 0 and q.least_score() == 0.0


def test_pq_overflow_and_bad_size(oracle):
    q = oracle.PriorityQueue(1)
    q.add(1, 1.0)
    with pytest.raises(IndexError):
        q.add(2, 2.0)
    with pytest.raises(ValueError):
        oracle.PriorityQueue(0)


def test_strict_log_is_fdlibm_within_an_ulp_of_libm(oracle):
    """The restated fdlibm log (Java's StrictMath.log, the LLR's Math.log up to an ulp): within one ulp of the C
    library's log everywhere it is finite, equal to it on the vast majority of inputs, IEEE special cases as Java
    specifies them (log(0) = -inf, log(negative) = NaN, log(inf) = inf, log(1) = 0)."""
    import math

    rng = np.random.default_rng(3)
    xs = np.concatenate([np.arange(1, 20001, dtype=np.float64), rng.integers(1, 1 << 62, 20000).astype(np.float64),
                         rng.random(20000) * 10, [5e-324, 1e-310, 0.5, 2.0, 10.0, 1 + 2 ** -30]])
    n_diff = 0
    for x in xs.tolist():
        a, b = oracle.strict_log(x), math.log(x)
        if a != b:
            n_diff += 1
            assert abs(a - b) <= math.ulp(b), (x, a, b)
    assert n_diff < 0.05 * len(xs)
    assert oracle.strict_log(0.0) == -math.inf and math.isnan(oracle.strict_log(-1.0))
    assert oracle.strict_log(math.inf) == math.inf and oracle.strict_log(1.0) == 0.0
    assert oracle.strict_log(2.0) == 0.6931471805599453 and oracle.strict_log(math.e) == 1.0
