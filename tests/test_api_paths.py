"""Module paths and names of the reference API that user code imports directly (collected from
the reference's unit tests): each resolves to the framework's implementation."""
import importlib

import numpy as np

import paddle_hackathon_amd as paddle

MODULES = ["static.amp", "static.amp.bf16", "nn.loss", "nn.layer.norm", "nn.layer.pooling", "nn.layer.activation",
           "framework.random", "tensor.stat", "tensor.array", "signal", "fluid.contrib.sparsity",
           "fluid.contrib.optimizer", "fluid.contrib.layers", "distributed.fleet.launch", "profiler.profiler",
           "fluid.dygraph.dygraph_to_static", "fluid.layers.utils", "incubate.nn.layer.fused_transformer",
           "distributed.fleet.meta_parallel.sharding.group_sharded_stage2",
           "distributed.fleet.meta_parallel.sharding.group_sharded_optimizer_stage2",
           "distributed.passes.pass_base", "distributed.fleet.elastic.manager", "fluid.incubate.data_generator",
           "fluid.layer_helper", "cost_model", "callbacks"]


def test_modules_import():
    for m in MODULES:
        importlib.import_module("paddle_hackathon_amd." + m)


def test_names():
    assert paddle.nn.loss.CrossEntropyLoss is paddle.nn.CrossEntropyLoss
    assert paddle.nn.layer.MaxPool2D is paddle.nn.MaxPool2D
    assert paddle.framework.ParamAttr is paddle.ParamAttr
    assert callable(paddle.framework.seed) and paddle.framework.get_default_dtype() == paddle.get_default_dtype()
    assert paddle.fluid.clip.GradientClipByGlobalNorm is paddle.nn.ClipGradByGlobalNorm
    assert paddle.fluid.framework.ParamBase is paddle.fluid.framework.EagerParamBase
    assert paddle.fluid.core.VarBase is paddle.Tensor
    np.testing.assert_allclose(paddle.tensor.math.inverse(paddle.to_tensor([[2.0, 0.0], [0.0, 4.0]])).numpy(),
                               [[0.5, 0.0], [0.0, 0.25]])
    assert paddle.tensor.random.gaussian([3, 2]).shape == [3, 2]


def test_signal_frame_overlap_add():
    x = paddle.to_tensor(np.arange(10, dtype="float32"))
    f = paddle.signal.frame(x, 4, 2)
    np.testing.assert_array_equal(f.numpy()[:, 1], [2, 3, 4, 5])
    np.testing.assert_array_equal(paddle.signal.overlap_add(f, 2).numpy(),
                                  [0, 1, 4, 6, 8, 10, 12, 14, 8, 9])


def test_tensor_array_and_switch_program():
    arr = paddle.tensor.create_array("float32")
    i = paddle.zeros([1], "int64")
    paddle.tensor.array_write(paddle.ones([2]), i, arr)
    assert int(paddle.tensor.array_length(arr).numpy().reshape(-1)[0]) == 1
    prog = paddle.static.Program()
    prev = paddle.fluid.framework.switch_main_program(prog)
    try:
        assert paddle.static.default_main_program() is prog
    finally:
        paddle.fluid.framework.switch_main_program(prev)


def test_distributed_optional_subsystems_loaded():
    """paddle.distributed's optional subsystems import together (a circular import there is
    swallowed by the package's guarded import and would silently drop them)"""
    d = paddle.distributed
    for n in ("spawn", "launch", "fleet", "split", "group_sharded_parallel", "ps", "auto_parallel", "passes",
              "shard_tensor", "shard_op", "ProcessMesh"):
        assert hasattr(d, n), n
