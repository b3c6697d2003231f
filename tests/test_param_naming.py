"""Parameter / accumulator names follow the reference's rules, and optimizer restores are strict.

Reference rules: Layer full names come from the global ``unique_name`` generator
(python/paddle/fluid/dygraph/layers.py:107); parameters are ``unique_name.generate(full_name +
".w" / ".b")`` (fluid/layer_helper_base.py:329); BatchNorm's running statistics are the layer's
next two ``.w`` names (nn/layer/norm.py:627-646); optimizer accumulators are
``unique_name.generate(param.name + "_" + acc)`` (optimizer/optimizer.py:636) and a missing one
is an assertion once a state dict was loaded (optimizer.py:656-659)."""
import numpy as np
import pytest

import paddle_hackathon_amd as paddle
from paddle_hackathon_amd.utils import unique_name


def _names(layer):
    return [p.name for p in layer.parameters()]


def test_layer_parameter_names_match_reference_rules():
    with unique_name.guard():
        lin = paddle.nn.Linear(3, 4)
        lin2 = paddle.nn.Linear(4, 2, bias_attr=False)
        conv = paddle.nn.Conv2D(3, 4, 3)
        bn = paddle.nn.BatchNorm2D(4)
        emb = paddle.nn.Embedding(10, 4)
        ln = paddle.nn.LayerNorm(4)
        convt = paddle.nn.Conv2DTranspose(4, 3, 3)
        named = paddle.nn.Linear(2, 2, weight_attr=paddle.ParamAttr(name="my_w"))
        assert _names(lin) == ["linear_0.w_0", "linear_0.b_0"]
        assert _names(lin2) == ["linear_1.w_0"]
        assert _names(conv) == ["conv2d_0.w_0", "conv2d_0.b_0"]
        assert _names(bn) == ["batch_norm2d_0.w_0", "batch_norm2d_0.b_0"]
        assert [b.name for b in bn.buffers()] == ["batch_norm2d_0.w_1", "batch_norm2d_0.w_2"]
        assert _names(emb) == ["embedding_0.w_0"]
        assert _names(ln) == ["layer_norm_0.w_0", "layer_norm_0.b_0"]
        assert _names(convt) == ["conv2d_transpose_0.w_0", "conv2d_transpose_0.b_0"]
        assert _names(named) == ["my_w", "linear_2.b_0"]
        assert paddle.create_parameter([2], "float32").name == "create_parameter_0.w_0"
        # structured state-dict keys are unchanged
        assert list(bn.state_dict().keys()) == ["weight", "bias", "_mean", "_variance"]


def test_static_builder_names_match_reference_rules():
    paddle.enable_static()
    try:
        with unique_name.guard():
            main, startup = paddle.static.Program(), paddle.static.Program()
            with paddle.static.program_guard(main, startup):
                x = paddle.static.data("x", [-1, 8], "float32")
                h = paddle.static.nn.fc(x, 6)
                paddle.static.nn.fc(h, 3)
            names = sorted(p.name for p in main.all_parameters())
            assert names == ["fc_0.b_0", "fc_0.w_0", "fc_1.b_0", "fc_1.w_0"]
    finally:
        paddle.disable_static()


def _train(model, opt, steps, seed):
    rng = np.random.RandomState(seed)
    for _ in range(steps):
        x = paddle.to_tensor(rng.randn(5, 3).astype("float32"))
        loss = (model(x) ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()


def test_adam_state_uses_reference_keys_and_resumes_step_for_step(tmp_path):
    with unique_name.guard():
        paddle.seed(1)
        a = paddle.nn.Linear(3, 4)
        opt_a = paddle.optimizer.Adam(0.05, parameters=a.parameters())
        _train(a, opt_a, 3, 0)
        sd = opt_a.state_dict()
        keys = sorted(k for k in sd if not k.startswith("@"))
        assert keys == sorted(f"linear_0.{p}_0_{acc}_0" for p in ("w", "b")
                              for acc in ("moment1", "moment2", "beta1_pow_acc", "beta2_pow_acc"))
        paddle.save(a.state_dict(), str(tmp_path / "m.pdparams"))
        paddle.save(sd, str(tmp_path / "m.pdopt"))
    # a fresh "process": a new generator gives the same names; the checkpoint holds reference keys
    with unique_name.guard():
        b = paddle.nn.Linear(3, 4)
        b.set_state_dict(paddle.load(str(tmp_path / "m.pdparams")))
        opt_b = paddle.optimizer.Adam(0.05, parameters=b.parameters())
        opt_b.set_state_dict(paddle.load(str(tmp_path / "m.pdopt")))
        _train(a, opt_a, 2, 7)
        _train(b, opt_b, 2, 7)
        for pa, pb in zip(a.parameters(), b.parameters()):
            np.testing.assert_allclose(pa.numpy(), pb.numpy(), rtol=1e-6, atol=1e-7)


def test_restore_with_other_generator_suffix_is_accepted():
    # the saving process had built another optimizer first: its keys end in _1
    with unique_name.guard():
        m = paddle.nn.Linear(3, 2)
        paddle.optimizer.Adam(0.1, parameters=m.parameters())._acc("moment1", m.weight)
        opt = paddle.optimizer.Adam(0.1, parameters=m.parameters())
        _train(m, opt, 1, 0)
        sd = opt.state_dict()
        assert "linear_0.w_0_moment1_1" in sd
    with unique_name.guard():
        m2 = paddle.nn.Linear(3, 2)
        opt2 = paddle.optimizer.Adam(0.1, parameters=m2.parameters())
        opt2.set_state_dict(sd)
        _train(m2, opt2, 1, 0)
        np.testing.assert_allclose(opt2._acc("moment2", m2.weight).numpy() > 0, True)


def test_missing_accumulator_raises_and_stray_keys_warn():
    with unique_name.guard():
        m = paddle.nn.Linear(3, 2)
        opt = paddle.optimizer.Adam(0.1, parameters=m.parameters())
        _train(m, opt, 1, 0)
        sd = {k: v for k, v in opt.state_dict().items() if "moment2" not in k or ".b_0" not in k}
    with unique_name.guard():
        m2 = paddle.nn.Linear(3, 2)
        opt2 = paddle.optimizer.Adam(0.1, parameters=m2.parameters())
        opt2.set_state_dict(sd)
        with pytest.raises(AssertionError, match="linear_0.b_0_moment2_0 should in state dict"):
            _train(m2, opt2, 1, 0)
    # state of a model whose parameters carry other names: reported, not silently dropped
    with unique_name.guard("other_"):
        m3 = paddle.nn.Linear(3, 2)
        opt3 = paddle.optimizer.Adam(0.1, parameters=m3.parameters())
        with pytest.warns(UserWarning, match="match no parameter"):
            opt3.set_state_dict(sd)
