"""ops/fallback.py: the hot-path fallback counter the GPU tests and the bench assert on
(tests/test_kernels_gpu.py::test_headline_paths_have_no_fallbacks)."""
import pytest

from paddle_hackathon_amd.ops import fallback


def test_counter_counts_and_resets(monkeypatch):
    monkeypatch.delenv("PHA_STRICT_NATIVE", raising=False)
    monkeypatch.delenv("PHA_FALLBACK_LOG", raising=False)
    fallback.reset()
    fallback.note("conv2d", "fp64")
    fallback.note("conv2d", "fp64")
    fallback.note("attention", "head dim 512")
    assert fallback.counts() == {"conv2d": 2, "attention": 1}
    assert fallback.total() == 3
    fallback.reset()
    assert fallback.total() == 0 and fallback.counts() == {}


def test_strict_native_raises(monkeypatch):
    monkeypatch.setenv("PHA_STRICT_NATIVE", "1")
    fallback.reset()
    with pytest.raises(RuntimeError, match="hot-path fallback: matmul"):
        fallback.note("matmul", "odd stride")
    fallback.reset()


def test_log_prints_each_reason_once(monkeypatch, capsys):
    monkeypatch.delenv("PHA_STRICT_NATIVE", raising=False)
    monkeypatch.setenv("PHA_FALLBACK_LOG", "1")
    fallback.reset()
    for _ in range(3):
        fallback.note("embedding", "fp32 table")
    err = capsys.readouterr().err
    assert err.count("[pha-fallback] embedding: fp32 table") == 1
    assert fallback.total() == 3
    fallback.reset()
