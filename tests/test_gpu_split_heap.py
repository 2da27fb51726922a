"""The two-pass rescoring's split heap pass (flink-cooccurrence_amd/csrc/cooc_stream.hip, k_rs_heap): rows longer
than a threshold are cut into segments whose own heaps keep, in order, the entries they could take, and the row's
heap replays only those.  The thresholds are shrunk (COOC_RS_SPLIT_LONG / _SEG / _CAP, read per call) so that the
long-rows log of test_c5_topk_long_rows_vs_oracle -- a hub with 45,000 near-equal partners (ties against the heap's
root) and one whose counts rise with the column (every later entry replaces the root) -- is split into dozens of
segments, and, with a cap of 16 kept entries, falls back to replaying whole rows.  The heaps must equal the
oracle's rescorer (ItemRowRescorer...java:195-241) bit for bit, as without the split.  Needs an MI355X."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("seg,cap", [("1024", "2048"), ("256", "2048"), ("1024", "16")])
def test_two_pass_split_long_rows_vs_oracle(pkg, oracle, torch_cuda, monkeypatch, seg, cap):
    monkeypatch.setenv("COOC_RS_TWO_PASS", "1")
    monkeypatch.setenv("COOC_RS_SPLIT_LONG", "1000")
    monkeypatch.setenv("COOC_RS_SPLIT_SEG", seg)
    monkeypatch.setenv("COOC_RS_SPLIT_CAP", cap)
    from tests.test_gpu_sparse import test_c5_topk_long_rows_vs_oracle

    test_c5_topk_long_rows_vs_oracle(pkg, oracle, torch_cuda)
