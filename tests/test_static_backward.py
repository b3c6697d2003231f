"""Per-op backward in the static Program (reference: python/paddle/fluid/backward.py:1141
_append_backward_ops_, :1381 append_backward) and the passes built on it: static recompute
(recompute_optimizer.py:20) and static AMP loss scaling (amp_optimizer.py:20). Each is checked
against the dygraph computation of the same weights."""
import numpy as np
import pytest

import paddle_hackathon_amd as paddle
from paddle_hackathon_amd.static import passes


@pytest.fixture
def static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def _mlp_program(w1, w2, checkpoints=False):
    main, startup = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, startup):
        x = paddle.static.data("x", [None, 4], "float32")
        y = paddle.static.data("y", [None, 1], "float32")
        W1 = paddle.static.create_parameter([4, 8], "float32", default_initializer=paddle.nn.initializer.Assign(w1))
        W2 = paddle.static.create_parameter([8, 1], "float32", default_initializer=paddle.nn.initializer.Assign(w2))
        h1 = paddle.tanh(paddle.matmul(x, W1))
        h2 = paddle.nn.functional.relu(h1 * 2.0 + h1)          # h1 feeds two ops: a sum of grads
        pred = paddle.matmul(h2, W2)
        loss = paddle.mean((pred - y) ** 2)
    return main, startup, x, y, W1, W2, h1, h2, loss


def _dygraph_grads(w1, w2, X, Y):
    """the same computation in torch fp64 autograd (independent of any framework-global state a
    previous test in the same worker may have left behind)"""
    import torch
    W1 = torch.tensor(w1, dtype=torch.float64, requires_grad=True)
    W2 = torch.tensor(w2, dtype=torch.float64, requires_grad=True)
    h1 = torch.tanh(torch.tensor(X, dtype=torch.float64) @ W1)
    h2 = torch.relu(h1 * 2.0 + h1)
    loss = ((h2 @ W2 - torch.tensor(Y, dtype=torch.float64)) ** 2).mean()
    loss.backward()
    return loss.item(), W1.grad.numpy().astype("float32"), W2.grad.numpy().astype("float32")


def _data():
    rng = np.random.RandomState(0)
    return (rng.randn(4, 8).astype("float32") * 0.5, rng.randn(8, 1).astype("float32") * 0.5,
            rng.randn(16, 4).astype("float32"), rng.randn(16, 1).astype("float32"))


def test_append_backward_emits_grad_ops(static_mode):
    w1, w2, X, Y = _data()
    main, startup, x, y, W1, W2, h1, h2, loss = _mlp_program(w1, w2)
    with paddle.static.program_guard(main, startup):
        pg = paddle.static.append_backward(loss)
    types = [op.type for op in main.global_block().ops]
    grad_types = [t for t in types if t.endswith("_grad")]
    assert "fill_constant" in types and "sum" in types
    assert {"matmul_grad", "tanh_grad", "relu_grad", "mean_grad"} <= set(grad_types), grad_types
    assert len(grad_types) >= 6
    names = dict((p.name, g.name) for p, g in pg)
    assert names[W1.name] == W1.name + "@GRAD" and names[W2.name] == W2.name + "@GRAD"
    assert any("@RENAME@" in v for v in main.global_block().vars)
    exe = paddle.static.Executor(paddle.CPUPlace())
    exe.run(startup)
    l, g1, g2 = exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss, pg[0][1], pg[1][1]])
    rl, r1, r2 = _dygraph_grads(w1, w2, X, Y)
    np.testing.assert_allclose(float(l), rl, rtol=1e-5)
    np.testing.assert_allclose(g1, r1, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(g2, r2, rtol=1e-5, atol=1e-6)


def test_minimize_with_grad_ops_trains(static_mode):
    w1, w2, X, Y = _data()
    main, startup, x, y, W1, W2, h1, h2, loss = _mlp_program(w1, w2)
    with paddle.static.program_guard(main, startup):
        paddle.optimizer.Adam(0.01).minimize(loss)
    types = [op.type for op in main.global_block().ops]
    assert types[-1] == "adam" and "matmul_grad" in types
    exe = paddle.static.Executor(paddle.CPUPlace())
    exe.run(startup)
    losses = [exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])[0].item() for _ in range(40)]
    assert losses[-1] < 0.5 * losses[0]


def test_static_recompute_matches(static_mode):
    """checkpoint at h1: the first segment runs without autograd state and is recomputed right
    before its grad ops; gradients equal the plain backward's"""
    w1, w2, X, Y = _data()
    main, startup, x, y, W1, W2, h1, h2, loss = _mlp_program(w1, w2)
    with paddle.static.program_guard(main, startup):
        pg = paddle.static.append_backward(loss, checkpoints=[h1])
    ops = main.global_block().ops
    assert any(op.attrs.get("recompute_of") for op in ops), "no recompute ops"
    assert any(op.attrs.get("no_grad") for op in ops)
    first_grad = next(i for i, op in enumerate(ops) if op.type.endswith("_grad") and op.attrs.get("fwd_type", "").endswith("tanh"))
    assert any(op.attrs.get("recompute_of") for op in ops[:first_grad])
    exe = paddle.static.Executor(paddle.CPUPlace())
    exe.run(startup)
    l, g1, g2 = exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss, pg[0][1], pg[1][1]])
    rl, r1, r2 = _dygraph_grads(w1, w2, X, Y)
    np.testing.assert_allclose(g1, r1, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(g2, r2, rtol=1e-5, atol=1e-6)


def test_static_amp_loss_scaling(static_mode):
    """loss@GRAD seeded with the scale, grads unscaled + finite-checked in one op, the dynamic
    scale update on device; an overflow skips nothing silently (found_inf is fetchable)"""
    w1, w2, X, Y = _data()
    main, startup, x, y, W1, W2, h1, h2, loss = _mlp_program(w1, w2)
    with paddle.static.program_guard(main, startup):
        pg = paddle.static.append_backward(loss)
        pg2, found_inf, state = passes.insert_loss_scaling(main, loss, pg, init_scale=1024.0, incr_every_n_steps=2)
    types = [op.type for op in main.global_block().ops]
    assert "check_finite_and_unscale" in types and "update_loss_scaling" in types
    exe = paddle.static.Executor(paddle.CPUPlace())
    exe.run(startup)
    g1, g2, inf = exe.run(main, feed={"x": X, "y": Y}, fetch_list=[pg2[0][1], pg2[1][1], found_inf])
    _, r1, r2 = _dygraph_grads(w1, w2, X, Y)
    np.testing.assert_allclose(g1, r1, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(g2, r2, rtol=1e-5, atol=1e-6)
    assert not bool(inf)
    exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])
    assert state["scale"].item() == 2048.0   # two good steps: scale doubled
