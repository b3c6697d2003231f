"""Fleet executor (reference fleet_executor/ carrier + interceptors, fleet_executor_utils TaskNode;
test_fleet_executor*.py): credit-based flow control, amplifier, Program-bodied compute tasks and
a two-rank pipeline whose cross-rank edge is a send/recv task pair."""
import numpy as np
import pytest
import torch

from dist_helper import run_dist

pytestmark = pytest.mark.timeout(120)


def _fe():
    from paddle_hackathon_amd.parallel.fleet_executor import FleetExecutor, TaskNode
    return FleetExecutor, TaskNode


def test_pipeline_with_credit_limit():
    FleetExecutor, TaskNode = _fe()
    n = 6
    src = TaskNode(0, n, node_type="Source", fn=lambda s: torch.tensor([float(s)]), task_id=1)
    mid = TaskNode(0, n, fn=lambda s, x: x * 2 + 1, task_id=2)
    snk = TaskNode(0, n, node_type="Sink", fn=lambda s, x: float(x[0]), task_id=3)
    src.add_downstream_task(2, 1)
    mid.add_upstream_task(1, 1)
    mid.add_downstream_task(3, 1)
    snk.add_upstream_task(2, 1)
    fe = FleetExecutor().init(num_micro_batches=n, task_nodes=[src, mid, snk])
    out = fe.run()
    assert out[3] == [2.0 * s + 1 for s in range(n)]
    # credit: the source is never more than buffer_size (1) steps ahead of what mid has consumed
    done = {1: 0, 2: 0, 3: 0}
    for tid, step in fe.trace:
        done[tid] = step + 1
        assert done[1] - done[2] <= 1 + 1 and done[2] - done[3] <= 1 + 1
    assert len(fe.trace) == 3 * n


def test_amplifier_and_program_task():
    import paddle_hackathon_amd as paddle
    FleetExecutor, TaskNode = _fe()
    paddle.enable_static()
    try:
        prog = paddle.static.Program()
        with paddle.static.program_guard(prog, paddle.static.Program()):
            x = paddle.static.data("x", [2], "float32")
            y = x * 3.0 + 1.0
    finally:
        paddle.disable_static()
    src = TaskNode(0, 4, node_type="Source", fn=lambda s: np.full(2, s, "float32"), task_id=10)
    comp = TaskNode(0, 4, program=prog, feed_names=["x"], fetch_list=[y], task_id=11)
    amp = TaskNode(0, 2, node_type="Sink", amplify=2, task_id=12,
                   fn=lambda s, xs: float(sum(float(v.numpy()[0]) for v in xs)))
    src.add_downstream_task(11)
    comp.add_upstream_task(10)
    comp.add_downstream_task(12, 2)
    amp.add_upstream_task(11, 2)
    out = FleetExecutor().init(num_micro_batches=4, task_nodes=[src, comp, amp]).run()
    # micro-batches 0..3 -> 3s+1 = 1, 4, 7, 10; the amplifier sums pairs
    assert out[12] == [5.0, 17.0]


def _two_rank(rank, world):
    import torch
    from paddle_hackathon_amd.parallel.fleet_executor import FleetExecutor, TaskNode
    n = 5
    src = TaskNode(0, n, node_type="Source", fn=lambda s: torch.full((3,), float(s)), task_id=1)
    st0 = TaskNode(0, n, fn=lambda s, x: (x + 1, x * 0 + s), task_id=2)
    st1 = TaskNode(1, n, fn=lambda s, xs: xs[0] * 10 + xs[1], task_id=3)
    snk = TaskNode(1, n, node_type="Sink", fn=lambda s, x: x.tolist(), task_id=4)
    src.add_downstream_task(2)
    st0.add_upstream_task(1)
    st0.add_downstream_task(3)
    st1.add_upstream_task(2)
    st1.add_downstream_task(4)
    snk.add_upstream_task(3)
    out = FleetExecutor().init(num_micro_batches=n, task_nodes=[src, st0, st1, snk],
                               task_id_to_rank={1: 0, 2: 0, 3: 1, 4: 1}).run()
    return {k: v for k, v in out.items()}


@pytest.mark.dist
def test_two_rank_pipeline_send_recv():
    r0, r1 = run_dist(_two_rank, 2)
    assert r0 == {}
    assert r1[4] == [[(s + 1) * 10.0 + s] * 3 for s in range(5)]


def test_failing_step_is_reported():
    FleetExecutor, TaskNode = _fe()

    def bad(s, x):
        if s == 2:
            raise ValueError("boom at 2")
        return x
    src = TaskNode(0, 4, node_type="Source", fn=lambda s: s, task_id=1)
    c = TaskNode(0, 4, fn=bad, task_id=2)
    src.add_downstream_task(2)
    c.add_upstream_task(1)
    with pytest.raises(ValueError, match="boom"):
        FleetExecutor().init(task_nodes=[src, c]).run()
