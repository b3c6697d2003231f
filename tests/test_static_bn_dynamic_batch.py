"""A static Program with a -1 batch dim whose BatchNorm layers train on 1 x 1 maps (ResNet-18 on
32 x 32 and 8 x 8 inputs). The recorded Variables keep -1 dims as size 1, and torch's batch-norm
check rejects N*H*W == 1 in training; the reference's InferMeta is shape-only
(phi/infermeta/multiary.cc:437), so the recording takes the op's shapes from probe-sized meta
runs instead (static/program.py ``_infer_meta_dynamic``). Losses match dygraph step for step."""
import copy

import numpy as np
import pytest

import paddle_hackathon_amd as paddle


@pytest.mark.parametrize("hw", [32, 8])
def test_resnet18_static_dynamic_batch_trains_like_dygraph(hw):
    paddle.seed(3)
    net = paddle.vision.models.resnet18(num_classes=10)
    ref = copy.deepcopy(net)
    rng = np.random.RandomState(0)
    batches = [(rng.rand(4, 3, hw, hw).astype("float32"), rng.randint(0, 10, [4, 1]).astype("int64"))
               for _ in range(3)]
    opt_d = paddle.optimizer.Momentum(0.01, parameters=ref.parameters())
    dy = []
    for x, y in batches:
        loss = paddle.nn.functional.cross_entropy(ref(paddle.to_tensor(x)), paddle.to_tensor(y))
        loss.backward()
        opt_d.step()
        opt_d.clear_grad()
        dy.append(float(loss))
    paddle.enable_static()
    try:
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            xv = paddle.static.data("x", [-1, 3, hw, hw], "float32")
            yv = paddle.static.data("y", [-1, 1], "int64")
            out = net(xv)
            assert list(out.shape) == [-1, 10]
            loss = paddle.nn.functional.cross_entropy(out, yv)
            paddle.optimizer.Momentum(0.01, parameters=net.parameters()).minimize(loss)
        exe = paddle.static.Executor()
        st = []
        for x, y in batches:
            lv, = exe.run(main, feed={"x": x, "y": y}, fetch_list=[loss])
            st.append(float(np.asarray(lv).reshape(-1)[0]))
        # another batch size through the same program
        exe.run(main, feed={"x": batches[0][0][:2], "y": batches[0][1][:2]}, fetch_list=[loss])
    finally:
        paddle.disable_static()
    np.testing.assert_allclose(st, dy, rtol=2e-4, atol=2e-5)


def test_instance_and_group_norm_dynamic_batch_record():
    paddle.enable_static()
    try:
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            x = paddle.static.data("x", [-1, 4, 1, 1], "float32")
            gn = paddle.nn.GroupNorm(2, 4)(x)
            bn = paddle.nn.BatchNorm2D(4)(x)
            assert list(gn.shape) == [-1, 4, 1, 1] and list(bn.shape) == [-1, 4, 1, 1]
        exe = paddle.static.Executor()
        g, b = exe.run(main, feed={"x": np.random.rand(3, 4, 1, 1).astype("float32")}, fetch_list=[gn, bn])
        assert g.shape == (3, 4, 1, 1) and b.shape == (3, 4, 1, 1)
    finally:
        paddle.disable_static()
