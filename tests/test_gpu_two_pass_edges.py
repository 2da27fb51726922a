"""Edge cases of the two-pass rescoring (flink-cooccurrence_amd/csrc/cooc_stream.hip: k_rs_score / k_rs_heap),
forced on small batch results in padded CSR (COOC_RS_TWO_PASS=1, read per call): one item, universes around
the 64-row chunk and 64-block boundaries, k = 1 and k = 1,024 (the largest heap it serves), k larger than any
row, exact and int-view scores, both planners.  Every heap against the oracle's rescorer
(ItemRowRescorer...java:195-241, via OracleStream) as in test_batch_topk_vs_rescorer.  Needs an MI355X."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

INT64_MAX = np.iinfo(np.int64).max


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("M,U,mean,k,exact,planner", [
    (1, 40, 3.0, 5, False, "auto"),
    (63, 300, 6.0, 1, False, "auto"),
    (65, 400, 8.0, 64, True, "auto"),
    (150, 800, 18.0, 7, False, "large"),
    (1000, 2000, 12.0, 300, False, "auto"),
    (3000, 3000, 20.0, 1024, True, "large"),
])
def test_two_pass_topk_edges_vs_rescorer(pkg, oracle, torch_cuda, monkeypatch, M, U, mean, k, exact, planner):
    from flink_cooccurrence_amd import datagen

    from tests._helpers import assert_topk_equal

    monkeypatch.setenv("COOC_RS_TWO_PASS", "1")
    up, it = datagen.small_log(1000 + M + k, U, M, mean)
    with pkg.CooccurrenceCore(n_items=M, output="csr", planner=planner) as core:
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
