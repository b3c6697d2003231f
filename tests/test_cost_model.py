"""paddle.cost_model (reference: python/paddle/fluid/tests/unittests/test_cost_model.py): per-op
times of a static program from core.CostModel().profile_measure and the static op benchmark table
(ours measured on MI355X)."""
import numpy as np

import paddle_hackathon_amd as paddle
from paddle_hackathon_amd.fluid import core


def test_profile_measure_empty_program():
    paddle.enable_static()
    try:
        cost = core.CostModel().profile_measure(paddle.static.Program(), paddle.static.Program(), "cpu", ["time"])
        assert cost.get_whole_time_ms() == 0
    finally:
        paddle.disable_static()


def test_profile_measure_program():
    paddle.enable_static()
    try:
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            # (the reference test builds X with paddle.ones; here an op with no Variable input is
            # folded to a constant at build time, so X is a fed data variable)
            data = paddle.static.data(name="X", shape=[16, 100], dtype="float32")
            hidden = paddle.static.nn.fc(data, 10)
            paddle.mean(hidden)
        cost = core.CostModel().profile_measure(main, startup, "cpu", ["time"],
                                                feed={"X": np.ones((16, 100), "float32")})
        n = cost.get_op_num()
        assert n == len(main.global_block().ops) and n >= 2
        times = [cost.get_op_time_ms(i) for i in range(n)]
        assert all(t > 0 for t in times)
        assert cost.get_whole_time_ms() >= sum(times)
    finally:
        paddle.disable_static()


def test_cost_model_demo_program_and_static_table():
    import os
    import pytest
    from paddle_hackathon_amd import cost_model
    if not os.path.exists(cost_model._TABLE):
        pytest.skip("static op table not generated yet (tools/gen_static_op_benchmark.py on the GPU)")
    cm = paddle.cost_model.CostModel()
    try:
        startup, main = cm.build_program()
        cost = cm.profile_measure(startup, main, "cpu")
        assert cost.get_whole_time_ms() > 0
    finally:
        paddle.disable_static()
    cm.static_cost_data()
    for op in ("abs", "conv2d", "matmul_v2", "softmax"):
        fwd = cm.get_static_op_time(op)
        bwd = cm.get_static_op_time(op, forward=False)
        assert float(fwd["op_time"]) > 0 and float(bwd["op_time"]) >= float(fwd["op_time"]), (op, fwd, bwd)
        assert "float32" in fwd["config"]
