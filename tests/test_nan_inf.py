"""FLAGS_check_nan_inf per-op scan (reference: paddle/fluid/eager/nan_inf_utils.cc; tests
python/paddle/fluid/tests/unittests/test_nan_inf.py — a NaN produced by an op aborts with
the op named)."""
import numpy as np
import pytest

import paddle_hackathon_amd as paddle


@pytest.fixture
def nan_flag():
    paddle.set_flags({"FLAGS_check_nan_inf": True, "FLAGS_check_nan_inf_level": 0})
    yield
    paddle.set_flags({"FLAGS_check_nan_inf": False, "FLAGS_check_nan_inf_level": 0})


def test_forward_op_named(nan_flag):
    x = paddle.to_tensor([1.0, 0.0])
    paddle.exp(x)  # finite: passes
    with pytest.raises(RuntimeError, match="`log`.*NaN"):
        paddle.log(x - 1.0)


def test_layer_output_named(nan_flag):
    lin = paddle.nn.Linear(2, 2)
    paddle.set_flags({"FLAGS_check_nan_inf": False})
    with paddle.no_grad():
        lin.weight.set_value(np.full([2, 2], np.inf, "float32"))
    paddle.set_flags({"FLAGS_check_nan_inf": True})
    with pytest.raises(RuntimeError, match="Inf"):
        lin(paddle.ones([1, 2]))


def test_backward_grad_checked(nan_flag):
    x = paddle.to_tensor([0.0, 1.0], stop_gradient=False)
    y = paddle.scale(x, 2.0)
    z = paddle.sqrt(y)  # finite forward; d sqrt / dy = inf at 0 -> flows into scale's output grad
    with pytest.raises(RuntimeError, match="scale_grad.*Inf"):
        paddle.sum(z).backward()


def test_level1_logs_only(nan_flag, caplog):
    paddle.set_flags({"FLAGS_check_nan_inf_level": 1})
    out = paddle.log(paddle.to_tensor([-1.0]))
    assert np.isnan(out.numpy()).all()
    assert any("NaN" in r.message for r in caplog.records)


def test_off_by_default():
    assert not paddle.get_flags("FLAGS_check_nan_inf")["FLAGS_check_nan_inf"]
    assert np.isnan(paddle.log(paddle.to_tensor([-1.0])).numpy()).all()
