"""Semi-auto parallel (reference tests: auto_parallel/test_engine_api.py, test_auto_parallel_*):
annotations lay tensors out as DTensors on a gloo mesh of 2 CPU ranks; Engine training with
Megatron-style column/row-sharded weights and with pure data parallelism matches a
single-process run of the same model."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dist_helper import run_dist  # noqa: E402

pytestmark = pytest.mark.dist


def _model_and_data(paddle):
    paddle.seed(3)
    model = paddle.nn.Sequential(paddle.nn.Linear(16, 32), paddle.nn.ReLU(), paddle.nn.Linear(32, 4))
    rng = np.random.default_rng(0)
    x = rng.standard_normal((40, 16)).astype(np.float32)
    y = (x[:, :4] * 0.5 - x[:, 4:8]).astype(np.float32)
    data = paddle.io.TensorDataset([paddle.to_tensor(x), paddle.to_tensor(y)])
    return model, data


def _single(paddle):
    model, data = _model_and_data(paddle)
    opt = paddle.optimizer.SGD(learning_rate=0.1, parameters=model.parameters())
    losses = []
    for xb, yb in paddle.io.DataLoader(data, batch_size=8):
        loss = paddle.nn.functional.mse_loss(model(xb), yb)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss.item()))
    return losses


def _tp_body(rank, world):
    import paddle_hackathon_amd as paddle
    import paddle_hackathon_amd.distributed as dist
    from paddle_hackathon_amd.distributed.auto_parallel import Engine, full_tensor_np
    ref = _single(paddle)
    model, data = _model_and_data(paddle)
    mesh = dist.ProcessMesh([0, 1], dim_names=["mp"])
    l1, l2 = model[0], model[2]
    w1_full = l1.weight.numpy().copy()
    dist.shard_tensor(l1.weight, dist_attr={"process_mesh": mesh, "dims_mapping": [-1, 0]})   # column split
    dist.shard_tensor(l1.bias, dist_attr={"process_mesh": mesh, "dims_mapping": [0]})
    dist.shard_tensor(l2.weight, process_mesh=mesh, shard_spec=["mp", None])                 # row split
    assert tuple(l1.weight._t.to_local().shape) == (16, 16) and tuple(l2.weight._t.to_local().shape) == (16, 4)
    assert np.array_equal(full_tensor_np(l1.weight), w1_full)
    eng = Engine(model)
    eng.prepare(paddle.optimizer.SGD(learning_rate=0.1, parameters=model.parameters()),
                loss=paddle.nn.functional.mse_loss, process_mesh=mesh)
    hist = eng.fit(data, batch_size=8, epochs=1)
    return ref, hist["loss"]


def test_engine_tensor_parallel_matches_single_process():
    for ref, got in run_dist(_tp_body, world=2):
        np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-6)


def _dp_body(rank, world):
    import paddle_hackathon_amd as paddle
    import paddle_hackathon_amd.distributed as dist
    from paddle_hackathon_amd.distributed.auto_parallel import Engine, Resharder, estimate_cost
    ref = _single(paddle)
    model, data = _model_and_data(paddle)
    mesh = dist.ProcessMesh([0, 1], dim_names=["dp"])
    eng = Engine(model)
    eng.prepare(paddle.optimizer.SGD(learning_rate=0.1, parameters=model.parameters()),
                loss=paddle.nn.functional.mse_loss, process_mesh=mesh)
    hist = eng.fit(data, batch_size=8, epochs=1)
    ev = eng.evaluate(data, batch_size=8)
    pred = eng.predict(data, batch_size=8)
    # reshard: a row-sharded tensor back to replicated
    t = paddle.to_tensor(np.arange(12, dtype=np.float32).reshape(4, 3))
    dist.shard_tensor(t, process_mesh=mesh, shard_spec=["dp", None])
    assert tuple(t._t.to_local().shape) == (2, 3)
    (full,) = Resharder([t], [{"process_mesh": mesh, "dims_mapping": [-1, -1]}]).reshard()
    assert np.array_equal(full._t.to_local().numpy(), np.arange(12, dtype=np.float32).reshape(4, 3))
    cost = estimate_cost(model, batch_size=8, process_mesh=mesh)
    assert cost["total"] > 0 and cost["params"] == 16 * 32 + 32 + 32 * 4 + 4
    return ref, hist["loss"], ev["loss"], len(pred), pred[0].shape


def test_engine_data_parallel_matches_single_process():
    for ref, got, ev_loss, n_pred, shp in run_dist(_dp_body, world=2):
        np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-6)
        assert ev_loss is not None and ev_loss < ref[0]
        assert n_pred == 5 and shp == (8, 4)


def test_annotation_only_without_process_group():
    import paddle_hackathon_amd as paddle
    import paddle_hackathon_amd.distributed as dist
    mesh = dist.ProcessMesh([[0, 1], [2, 3]], dim_names=["dp", "mp"])
    assert mesh.topology == [2, 2] and mesh.processes == [0, 1, 2, 3] and mesh.ndim == 2
    w = paddle.create_parameter([8, 4], "float32")
    dist.shard_tensor(w, process_mesh=mesh, shard_spec=[None, "mp"])
    assert w.dist_attr["dims_mapping"] == [-1, 1] and w.shape == [8, 4]
    with pytest.raises(ValueError):
        dist.shard_tensor(w, dist_attr={"process_mesh": mesh, "dims_mapping": [0, 0]})
    add = dist.shard_op(paddle.add, process_mesh=mesh, in_shard_specs=[["dp", None], None])
    out = add(paddle.ones([4, 4]), paddle.ones([4, 4]))
    assert float(out.sum().item()) == 32.0
